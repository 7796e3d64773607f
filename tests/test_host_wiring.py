"""Host-side decisions of the GATModel wiring fused into the layers (CPU, no kernel calls): which
layers fold their Linear skip into the projection GEMM, which apply the next layer's input
dropout in their epilogue, and the skip-fold / dropout-fuse switches. Reference wiring:
`models/GATModel.py:64-116` (skip construction) and `:128-149` (dropout, skip-add, ELU)."""
import pytest

from gatx.config import data_config


def _model(name, **over):
    import gatx
    cfg = dict(data_config[name])
    cfg.update(over)
    return gatx.GATModel(**cfg)


def test_skip_modules_follow_the_reference():
    from torch import nn
    pat = _model("PATTERN")   # 3 -> 48 -> 96 -> 48 -> 1: every skip a Linear
    assert all(isinstance(s, nn.Linear) for s in pat.skip_layer_list)
    assert [tuple(s.weight.shape) for s in pat.skip_layer_list] == [(48, 3), (96, 48), (48, 96),
                                                                      (1, 48)]
    ppi = _model("PPI")       # layer 1's skip is 1024 -> 1024: Identity
    assert len(ppi.skip_layer_list) == 1 and isinstance(ppi.skip_layer_list[0], nn.Identity)


@pytest.mark.parametrize("name,expected", [
    ("Cora", [True, False]),       # layer 0 (1433 -> 8x8) feeds layer 1's dropout
    ("Pubmed", [True, False]),
    ("Citeseer", [True, False]),
    ("PPI", [False, True, False]),    # layer 1 has a skip (reads the undropped input), so layer
                                      # 0 does not drop for it; layer 1 feeds layer 2's dropout
    ("PATTERN", [False, False, False, False]),   # every layer has a skip
])
def test_next_layer_dropout_fusion_decisions(name, expected):
    m = _model(name)
    assert [m._fuse_next_dropout(i) for i in range(m.num_layers)] == expected


def test_dropout_fuse_switch(monkeypatch):
    from gatx import tuning
    tuning.set(dropout_fuse=0)
    m = _model("Cora")
    assert not any(m._fuse_next_dropout(i) for i in range(m.num_layers))


def test_output_dropout_needs_an_edge_pass_epilogue():
    from gatx.functional import fuses_output_dropout, use_reassociation, LayerShape
    # PPI layer 0 (50 -> 4 x 256) is reassociated: no fused output dropout
    assert use_reassociation(LayerShape(4, 256, 50, True, False))
    assert not fuses_output_dropout(4, 256, 50, True)
    # head-mean layers and wide inputs take the direct edge pass
    assert fuses_output_dropout(6, 121, 1024, False)
    assert fuses_output_dropout(8, 8, 1433, True)


def test_reference_wiring_flag_defaults_to_fused():
    m = _model("PPI")
    assert m.fuse_wiring is True


def test_split_gemm_kernel_choices(monkeypatch):
    """Which GEMMs take the pre-split weight planes (gemm_f16p) and the f16x3 weight gradient
    (gemm_f16rc): PPI's projection / g_x shapes do, small or unaligned weights and wide weight
    gradients do not, and tuning f16p=0 turns both off (no GPU call: the library only reports its
    arithmetic mode)."""
    from gatx import functional as gf
    from gatx._lib import lib
    from gatx import tuning
    lib.gatx_set_gemm_mode(2)
    try:
        assert gf.use_weight_planes(1032, 1024, 44900)        # PPI L1 projection
        assert gf.use_weight_planes(1024, 1032, 44900)        # PPI L1 g_x (W_aug^T)
        assert not gf.use_weight_planes(48, 1024, 44900)      # small output
        assert not gf.use_weight_planes(1032, 50, 44900)      # k not a multiple of 4
        assert not gf.use_weight_planes(1032, 1024, 100)      # few rows
        assert gf.use_wgrad_f16(1032, 1024, 44900)
        assert not gf.use_wgrad_f16(4096, 1024, 44900)        # beyond the 2048 column maxima
        assert not gf.use_wgrad_f16(1032, 50, 44900)
        assert lib.gatx_gemm_layout_mode(1, 1) == 2 and lib.gatx_gemm_layout_mode(0, 0) == 2
        assert lib.gatx_gemm_layout_mode(1, 0) == 1
        tuning.set(f16p=0)
        assert not gf.use_weight_planes(1032, 1024, 44900)
        assert not gf.use_wgrad_f16(1032, 1024, 44900)
        lib.gatx_set_gemm_mode(1)
        tuning.reset()
        assert not gf.use_weight_planes(1032, 1024, 44900)    # x3 arithmetic: no planes
        assert lib.gatx_gemm_layout_mode(1, 1) == 1
    finally:
        lib.gatx_set_gemm_mode(2)
        tuning.reset()


def test_lds_pass_bounded_by_its_index_limits():
    """The LDS-staged pass is chosen only inside the kernels' index limits: E' < 2^28 (32-bit
    record byte offsets) and N < 2^25 (64 src in an int32); past them the layer takes the
    L2-gather pass instead of raising in gatx_edge_lds_forward (no GPU call: a stand-in graph)."""
    from gatx import functional as gf
    from gatx.functional import LayerShape

    class FakeGraph:
        def __init__(self, edge_bound, num_nodes):
            self.edge_bound, self.num_nodes = edge_bound, num_nodes

        def lds_blocks(self, max_rows, side=False):
            return ("segs", "count", 20)

    sh = LayerShape(4, 256, 1024, True, False)
    assert gf.lds_blocks(FakeGraph(1 << 21, 44900), sh) is not None
    assert gf.lds_blocks(FakeGraph((1 << 28) - 1, 44900), sh) is not None
    assert gf.lds_blocks(FakeGraph(1 << 28, 44900), sh) is None
    assert gf.lds_blocks(FakeGraph(1 << 21, (1 << 25) - 1), sh) is not None
    assert gf.lds_blocks(FakeGraph(1 << 21, 1 << 25), sh) is None
    assert gf.lds_blocks(FakeGraph(1 << 10, 100), sh) is None    # below lds_min_edges


def test_edge_count_promise_bound_to_tensor_and_version():
    """expect_num_edges binds its promise to the tensor object at its current version: an in-place
    rewrite, or another tensor at the same address, finds no promise (CPU tensors: the lookup
    reads only identity, shape and version)."""
    import torch
    from gatx.graph import expect_num_edges, _hint_lookup
    ei = torch.zeros(2, 10, dtype=torch.int64)
    expect_num_edges(ei, 5, True, 13)
    assert _hint_lookup(ei, 5, True) == 13
    assert _hint_lookup(ei, 6, True) is None
    alias = ei.view(2, 10)             # same storage and shape, another tensor object
    assert _hint_lookup(alias, 5, True) is None
    ei.add_(1)                         # rewritten in place
    assert _hint_lookup(ei, 5, True) is None
    expect_num_edges(ei, 5, True, 14)
    assert _hint_lookup(ei, 5, True) == 14
    expect_num_edges(ei, 5, True, None)
    assert _hint_lookup(ei, 5, True) is None
