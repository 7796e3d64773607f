"""The host path's tuning switches, set explicitly in-process (never read from the environment,
so an inherited environment cannot change which kernels or dataflow run).

Every switch selects between two correct, GPU-tested implementations of the same result (or a
threshold of one); the defaults are the measured-best choices:

  f16p            1     pre-split fp16 weight planes for the f16x3 projection / g_x GEMMs and the
                        f16x3 weight gradient (0: the in-loop split kernels)
  heads_per_item  0     heads per edge-pass work item (0: edge_heads_per_item's rule)
  mean_heads      0     head-group size of head-mean layers (0: the rule)
  edge_chunk      2048  destination nodes per (chunk, head group) sweep of the edge passes
  hub_edges       8192  forward hub splitting: segments longer than this run in pieces (0: off)
  hub_min_edges   2^22  ... only in graphs of more input edges than this
  bwd_hub_edges   65536 backward hub splitting threshold (0: off)
  bwd_hubs        1     backward hub splitting on / off
  reassoc         1     first-layer reassociation (aggregate x rows, then project) when it pays
  fused_scores    1     node scores reduced in the projection GEMM's epilogue
  dropout_fuse    1     the next layer's input dropout in this layer's edge-pass epilogue
  skip_fold       1     GATModel's Linear skips folded into the projection GEMM
  edge_lds        1     concat layers on graphs cut into node blocks of <= 2304 nodes: the
                        LDS-staged edge pass (csrc/edge_lds.hip) instead of the L2-gather one
  edge_lds_mean   1     head-mean layers take it too (gatx_edge_lds_mean_forward: every head
                        staged in turn, the mean kept in registers), round 6
  edge_lds_bwd    1     the backward's source pass of a concat layer (F % 4 == 0) on such graphs:
                        transposed records (gatx_edge_records_src) + the same LDS walk over go's
                        rows (0: the L2-gather source pass), round 6
  side_stream     0     short independent launches (node blocks, GATModel's non-final alpha
                        passes) on a second stream, under the projection GEMM. Off since round 6:
                        with the windowed node-block build (~21 us serial) the fork / join gaps
                        of a replayed graph (~5-9 us each) and the alpha pass sharing CUs with the
                        output projection cost more than the overlap saved (PPI fwd 1.427 serial
                        vs 1.435 ms, interleaved A/B, round 6 session 1; the run's files were
                        lost with that session's container)
  lds_min_edges   2^18  edge_lds / side_stream only on graphs of at least this many edges
                        (edge_index' bound): below it a step is launch-bound, and the extra
                        launches and cross-queue joins cost more than they save (PATTERN G=8)

    import gatx
    with gatx.tuning.override(edge_chunk=2245):   # or gatx.tuning.set(...) / reset()
        model(x, edge_index)
"""
from __future__ import annotations

from contextlib import contextmanager

DEFAULTS = {
    "f16p": 1,
    "heads_per_item": 0,
    "mean_heads": 0,
    "edge_chunk": 2048,
    "hub_edges": 8192,
    "hub_min_edges": 1 << 22,
    "bwd_hub_edges": 65536,
    "bwd_hubs": 1,
    "reassoc": 1,
    "fused_scores": 1,
    "dropout_fuse": 1,
    "skip_fold": 1,
    "edge_lds": 1,
    "edge_lds_mean": 1,
    "edge_lds_bwd": 1,
    "side_stream": 0,
    "lds_min_edges": 1 << 18,
}

_current = dict(DEFAULTS)


def get(name: str) -> int:
    return _current[name]


def set(**switches) -> None:  # noqa: A001  (module-level API: gatx.tuning.set)
    for k, v in switches.items():
        if k not in DEFAULTS:
            raise KeyError(f"gatx.tuning: unknown switch {k!r} (known: {sorted(DEFAULTS)})")
        _current[k] = int(v)


def reset() -> None:
    _current.clear()
    _current.update(DEFAULTS)


def current() -> dict:
    return dict(_current)


@contextmanager
def override(**switches):
    saved = dict(_current)
    try:
        set(**switches)
        yield
    finally:
        _current.clear()
        _current.update(saved)


def parse(assignments) -> dict:
    """["edge_chunk=2245", ...] -> {"edge_chunk": 2245} (bench.py --tune)."""
    out = {}
    for a in assignments or []:
        k, _, v = a.partition("=")
        if k not in DEFAULTS or not v:
            raise ValueError(f"gatx.tuning: bad assignment {a!r} (known: {sorted(DEFAULTS)})")
        out[k] = int(v, 0)
    return out
