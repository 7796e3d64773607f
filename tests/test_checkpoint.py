"""The weights-only checkpoint reader (gatx.checkpoint.read_state_dict) on the reference's trained
checkpoints (`checkpoints/*.ckpt`, loaded by `data_utils.py:36-47`), checked against an
independent parse: the raw little-endian storages in the zip, and the shapes / byte sizes /
parameter counts SURVEY.md §8(c) lists. Plus malformed archives, which must raise, never read
out of bounds. CPU only; skipped where the reference tree is absent (the GPU box)."""
import io
import os
import zipfile

import numpy as np
import pytest

from gatx.checkpoint import _check_view, read_state_dict

CKPT = "/root/reference/checkpoints"
need_ref = pytest.mark.skipif(not os.path.isdir(CKPT), reason="reference checkpoints absent")

# SURVEY.md §8(c) "Reading trained weights without unpickling"
SHAPES = {
    "Cora": {"gat_layer_list.0.W.weight": (64, 1433), "gat_layer_list.0.a.weight": (8, 128),
             "gat_layer_list.1.W.weight": (7, 64), "gat_layer_list.1.a.weight": (1, 14)},
    "Citeseer": {"gat_layer_list.0.W.weight": (64, 3703), "gat_layer_list.0.a.weight": (8, 128),
                 "gat_layer_list.1.W.weight": (6, 64), "gat_layer_list.1.a.weight": (1, 12)},
    "Pubmed": {"gat_layer_list.0.W.weight": (64, 500), "gat_layer_list.0.a.weight": (8, 128),
               "gat_layer_list.1.W.weight": (24, 64), "gat_layer_list.1.a.weight": (8, 48)},
    "PATTERN": {"gat_layer_list.0.W.weight": (48, 3), "gat_layer_list.1.W.weight": (96, 48),
                "gat_layer_list.2.W.weight": (48, 96), "gat_layer_list.3.W.weight": (1, 48),
                "gat_layer_list.0.a.weight": (4, 96), "gat_layer_list.1.a.weight": (4, 192),
                "gat_layer_list.2.a.weight": (4, 96), "gat_layer_list.3.a.weight": (1, 2),
                "skip_layer_list.0.weight": (48, 3), "skip_layer_list.1.weight": (96, 48),
                "skip_layer_list.2.weight": (48, 96), "skip_layer_list.3.weight": (1, 48)},
}
PARAM_COUNTS = {"Cora": 93198, "PATTERN": 20354}


def _raw_storages(path):
    """{storage key: fp32 array} straight from the zip members, no pickle involved."""
    with zipfile.ZipFile(path) as zf:
        root = zf.namelist()[0].split("/")[0]
        return {n.rsplit("/", 1)[1]: np.frombuffer(zf.read(n), dtype="<f4")
                for n in zf.namelist() if n.startswith(f"{root}/data/")}


@need_ref
@pytest.mark.parametrize("name", sorted(SHAPES))
def test_reader_matches_raw_storages(name):
    path = f"{CKPT}/{name}-100epochs.ckpt"
    sd = read_state_dict(path)
    for k, shp in SHAPES[name].items():
        assert sd[k].shape == shp and sd[k].dtype == np.float32, k
        assert sd[k].flags.c_contiguous
    params = {k: v for k, v in sd.items() if not k.startswith("loss_fn.")}
    assert set(params) == set(SHAPES[name])
    if name in PARAM_COUNTS:
        assert sum(v.size for v in params.values()) == PARAM_COUNTS[name]
    # every tensor is exactly one whole raw storage (offset 0, contiguous) in this archive:
    # match each to its storage by bytes, independent of the pickle walk
    raw = _raw_storages(path)
    for k, v in params.items():
        hits = [s for s in raw.values() if s.size == v.size and np.array_equal(s, v.reshape(-1))]
        assert hits, k
    if name == "Cora":   # Cora W = 366 848 B = 64 x 1433 x 4
        assert sd["gat_layer_list.0.W.weight"].nbytes == 366848
    if name == "PATTERN":
        # the checkpoint predates pattern_gat.py:13's 1/0.1765 ("previously [4.65]")
        assert np.allclose(sd["loss_fn.pos_weight"], 4.65)


def _rewrite(path, mutate):
    """A copy of the archive with member bytes changed by mutate(name, bytes) -> bytes."""
    buf = io.BytesIO()
    with zipfile.ZipFile(path) as src, zipfile.ZipFile(buf, "w") as dst:
        for n in src.namelist():
            dst.writestr(n, mutate(n, src.read(n)))
    buf.seek(0)
    return buf


@need_ref
def test_truncated_storage_raises(tmp_path):
    path = f"{CKPT}/Cora-100epochs.ckpt"
    # cut the largest storage (W of layer 0) in half: its view would reach past the buffer
    with zipfile.ZipFile(path) as zf:
        big = max((n for n in zf.namelist() if "/data/" in n), key=lambda n: zf.getinfo(n).file_size)
    bad = _rewrite(path, lambda n, b: b[: len(b) // 2] if n == big else b)
    p = tmp_path / "bad.ckpt"
    p.write_bytes(bad.read())
    with pytest.raises(ValueError, match="storage holds"):
        read_state_dict(str(p))


@need_ref
def test_tampered_pickle_raises(tmp_path):
    path = f"{CKPT}/PATTERN-100epochs.ckpt"
    # an unknown opcode in the pickle stream (a hostile file) is refused, never executed
    bad = _rewrite(path, lambda n, b: (b[:2] + b"\x93" + b[2:]) if n.endswith("data.pkl") else b)
    p = tmp_path / "bad.ckpt"
    p.write_bytes(bad.read())
    with pytest.raises(Exception):
        read_state_dict(str(p))


def test_view_bounds():
    _check_view("t", 12, 0, (3, 4), (4, 1))
    _check_view("t", 12, 0, (0, 4), (4, 1))
    for args in [(12, 1, (3, 4), (4, 1)), (12, 0, (4, 4), (4, 1)), (12, -1, (2,), (1,)),
                 (12, 0, (2, 2), (-1, 1)), (12, 0, (3,), (1, 1)), (12, 0, (-2,), (1,))]:
        with pytest.raises(ValueError):
            _check_view("t", *args)
