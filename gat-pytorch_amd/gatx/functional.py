"""Autograd wiring of the fused GAT layer: forward = projection GEMM (+ per-node attention scores)
-> global max -> fused edge pass; backward = dst pass -> max() backward -> src pass -> two GEMMs
-> weight-gradient fix-ups. All device work is in libgatx.so (csrc/); this file only allocates
tensors from torch's caching allocator and launches on torch's current stream.

Reference: models/gat_layer.py:42-140 (forward); its autograd is restated in closed form in
SURVEY.md §8(a) a14 and oracle/gat_oracle.py:gat_layer_backward.
"""
from __future__ import annotations

import ctypes
from contextlib import contextmanager

import torch

from . import tuning
from ._lib import ARGMAX_CAP, call, lib, ptr, stream, version
from .graph import Graph, join_side


class KernelTimer:
    """Optional HIP-event bracketing of the forward's launches (bench.py's live per-kernel
    timing). Events are recorded on torch's current stream — the stream every gatx launch uses."""

    def __init__(self):
        self.records = []   # (phase, info, start_event, end_event)

    def span(self, phase, info):
        timer = self

        class _Span:
            def __enter__(self):
                self.s = torch.cuda.Event(enable_timing=True)
                self.e = torch.cuda.Event(enable_timing=True)
                self.s.record()
                return self

            def __exit__(self, *exc):
                self.e.record()
                timer.records.append((phase, info, self.s, self.e))
                return False
        return _Span()

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for phase, info, s, e in self.records:
            out.setdefault(phase, []).append((info, s.elapsed_time(e)))
        return out


_timer: "KernelTimer | None" = None


def set_kernel_timer(t):
    global _timer
    _timer = t


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def _span(phase, info):
    return _timer.span(phase, info) if _timer is not None else _Null()


def _round4(v: int) -> int:
    return (v + 3) // 4 * 4


def _require(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"gatx: {name} must be on the HIP device (no CPU path)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"gatx: {name} must be float32, got {t.dtype}")


class LayerShape:
    def __init__(self, num_heads: int, out_features: int, in_features: int, concat: bool,
                 const_attention: bool):
        self.NH, self.F, self.F_in = num_heads, out_features, in_features
        self.concat, self.const = bool(concat), bool(const_attention)
        self.Fp = _round4(out_features)
        self.Dp = self.NH * self.Fp
        self.H2 = 0 if self.const else 2 * self.NH
        self.K_aug = self.Dp + self.H2
        self.ldg = _round4(self.K_aug)
        self.out_cols = self.NH * self.F if self.concat else self.F
        # GATModel's Linear skip folded into the projection (skip_weight=): its out_cols rows
        # follow W_aug's K_aug rows (0: no folded skip)
        self.skip_cols = 0
        # derived weights (W_aug, padded W) may be cached: decided by gat_layer() before
        # autograd.Function.forward, inside which grad mode is always off (see _cacheable)
        self.cache_weights = True


_MAX_WS = {}


def _max_ws(dev):
    """Per-device scratch for the max pre-pass partials (reused: stream-ordered)."""
    t = _MAX_WS.get(dev)
    if t is None:
        t = torch.empty(lib.gatx_attention_max_workspace_bytes(), dtype=torch.uint8, device=dev)
        _MAX_WS[dev] = t
    return t


_WAUG_CACHE: "OrderedDict" = None


def gemm_workspace(M: int, N: int, K: int, dev):
    """(pointer, bytes) of the tail-split workspace gatx_gemm_f32 / gatx_projection_gemm may
    use for an (M x K) . (K x N) product (cached allocator; None when this shape needs none)."""
    nb = lib.gatx_gemm_workspace_bytes(M, N, K)
    if nb == 0:
        return None, 0
    return ptr(torch.empty(nb, dtype=torch.uint8, device=dev)), nb


_WPAD_CACHE: "OrderedDict" = None


def _cacheable(*params) -> bool:
    """Derived-weight caches are used only when no gradient flows to the weights (eval /
    no_grad / inference): a training step rebuilds them from the live parameters every forward,
    so in-place updates that bypass the version counter (`p.data.mul_()`, EMA / weight averaging
    through `.data`) can never leave a stale copy in the gradient path. In no-grad use the key is
    (storage, version counter): such a `.data` update between two eval forwards is not seen —
    call `clear_weight_cache()` after one (load_state_dict and optimizer steps bump the version
    and are seen)."""
    if torch.is_grad_enabled() and any(p is not None and p.requires_grad for p in params):
        return False
    return True


def clear_weight_cache():
    """Drop every cached derived weight (W_aug, padded W); see _cacheable."""
    if _WAUG_CACHE is not None:
        _WAUG_CACHE.clear()
    if _WPAD_CACHE is not None:
        _WPAD_CACHE.clear()


def padded_weight(W, ld: int, use_cache: bool = True):
    """W (rows x F_in) copied into rows of `ld` floats (zero tail, gatx_pad_rows) so GEMMs can
    read it as float4 rows; cached on the parameter's identity and version (see _cacheable)."""
    global _WPAD_CACHE
    from collections import OrderedDict
    if W.size(1) == ld:
        return W
    if _WPAD_CACHE is None:
        _WPAD_CACHE = OrderedDict()
    key = (W.data_ptr(), version(W), tuple(W.shape), W.device, ld)
    hit = _WPAD_CACHE.get(key) if use_cache else None
    if hit is not None:
        _WPAD_CACHE.move_to_end(key)
        return hit[1]
    Wp = torch.empty((W.size(0), ld), dtype=torch.float32, device=W.device)
    call("gatx_pad_rows", ptr(W), W.size(0), W.size(1), W.size(1), ptr(Wp), ld, stream())
    if use_cache:
        _WPAD_CACHE[key] = (W, Wp)
        while len(_WPAD_CACHE) > 16:
            _WPAD_CACHE.popitem(last=False)
    return Wp


def augmented_weight(W, a, sh: "LayerShape", skip_W=None):
    """W_aug = [W padded per head; A_src W; A_dst W] (gatx_prepare_weights), followed, when
    GATModel's Linear skip is folded in (skip_W), by its out_cols rows W_skip_eff
    (gatx_skip_weight_rows: the head mean folded into the weight for a head-mean layer). Rebuilt
    every training forward; in no-grad use cached on the parameters' identity and version
    counters, so inference reuses it across steps while load_state_dict / optimizer steps rebuild
    it (see _cacheable for the `.data` caveat)."""
    global _WAUG_CACHE
    from collections import OrderedDict
    if _WAUG_CACHE is None:
        _WAUG_CACHE = OrderedDict()
    use_cache = sh.cache_weights
    key = (W.data_ptr(), version(W), tuple(W.shape), W.device,
           a.data_ptr() if a is not None else 0, version(a) if a is not None else -1,
           sh.NH, sh.F, sh.concat if skip_W is not None else None,
           skip_W.data_ptr() if skip_W is not None else 0,
           version(skip_W) if skip_W is not None else -1)
    hit = _WAUG_CACHE.get(key) if use_cache else None
    if hit is not None:
        _WAUG_CACHE.move_to_end(key)
        return hit[2]
    C = sh.out_cols if skip_W is not None else 0
    waug_floats = lib.gatx_prepare_weights_skip_floats(sh.NH, sh.F, sh.F_in, int(a is not None), C)
    W_aug = torch.empty(waug_floats, dtype=torch.float32, device=W.device)
    with _span("prepare_weights", (sh.NH, sh.F, sh.F_in)):
        call("gatx_prepare_weights_skip", ptr(W), ptr(a), sh.NH, sh.F, sh.F_in, ptr(skip_W),
             1 if sh.concat else sh.NH, C, ptr(W_aug), stream())
    if use_cache:
        # holding W / a / skip_W pins their storage (no pointer reuse)
        _WAUG_CACHE[key] = (W, a, W_aug, skip_W)
        while len(_WAUG_CACHE) > 16:
            _WAUG_CACHE.popitem(last=False)
    return W_aug


def use_weight_planes(rows: int, k: int, m: int) -> bool:
    """Whether a GEMM with this weight operand takes the pre-split f16x3 kernel (gemm_f16p.hip):
    the f16x3 arithmetic, float4-aligned rows, and outputs big enough for its 256 x 256 tiles (the
    library makes the final choice; planes it does not use cost one small build per weight
    version; gatx_weight_planes_bytes is 0 for a weight too tall for the planes' header, which
    then takes the in-loop split kernel). tuning f16p=0: never build them."""
    if tuning.get("f16p") == 0 or lib.gatx_get_gemm_mode() != 2:
        return False
    return (k % 4 == 0 and rows >= 256 and m >= 256
            and lib.gatx_weight_planes_bytes(rows, k) > 0)


def use_wgrad_f16(M: int, N: int, K: int) -> bool:
    """Whether the weight gradient G_aug^T x (M = K_aug rows, N = F_in, K = nodes) takes the
    row-contiguous f16x3 kernel (gemm_f16p.hip, scales from G_aug's exact column maxima): the
    f16x3 arithmetic and an output its 256 x 256 tiles cover (the library decides finally; the
    statistics pass is then only wasted work). tuning f16p=0: never."""
    if tuning.get("f16p") == 0 or lib.gatx_get_gemm_mode() != 2:
        return False
    return M >= 256 and N >= 256 and M <= 2048 and N % 4 == 0


def build_weight_planes(W, rows: int, k: int, ld: int):
    """fp16 planes of the weight W (rows x k, row stride ld) for gatx_gemm_planes: one 256-byte
    aligned buffer (header + planes), built on the current stream."""
    nb = lib.gatx_weight_planes_bytes(rows, k)
    buf = torch.empty(nb + 256, dtype=torch.uint8, device=W.device)
    off = (-ptr(buf)) % 256
    planes = buf[off:off + nb]
    call("gatx_weight_planes", ptr(W), rows, k, ld, ptr(planes), stream())
    return planes


def projection_planes(W_aug, sh: "LayerShape", N: int):
    """The planes of the projection weight W_aug ([K_aug + C] x F_in), cached beside W_aug (same
    key, same lifetime) in no-grad use, rebuilt with it in training; None when the pre-split
    kernel would not take the GEMM."""
    rows = sh.K_aug + sh.skip_cols
    if not use_weight_planes(rows, sh.F_in, N):
        return None
    if sh.cache_weights and _WAUG_CACHE is not None:
        for key, val in _WAUG_CACHE.items():
            if val[2] is W_aug:
                if len(val) > 4:
                    return val[4]
                planes = build_weight_planes(W_aug, rows, sh.F_in, sh.F_in)
                _WAUG_CACHE[key] = val[:4] + (planes,)
                return planes
    return build_weight_planes(W_aug, rows, sh.F_in, sh.F_in)


_SIDE_ALPHA = [False]


@contextmanager
def side_alpha(on: bool):
    """Within: a layer's alpha pass (and its max() tie records) is launched on the side stream,
    forked after the edge pass, so it runs under the next layer's projection GEMM; the next
    layer joins it after launching that GEMM, and GATModel joins before returning (the alphas
    and tie records are read by nothing in between). Only GATModel sets it, for all but its last
    layer."""
    prev = _SIDE_ALPHA[0]
    _SIDE_ALPHA[0] = on
    try:
        yield
    finally:
        _SIDE_ALPHA[0] = prev


def _alpha_pass(graph: Graph, S, M_ord, den, sh: "LayerShape", alpha, argmax, dev):
    """_attention_alpha on the current stream, or forked onto the side stream (side_alpha)."""
    if not (_SIDE_ALPHA[0] and tuning.get("side_stream")
            and graph.edge_bound >= tuning.get("lds_min_edges")):
        with _span("attention_alpha", (graph.edge_bound, sh.NH)):
            _attention_alpha(graph, S, M_ord, den, sh, alpha, argmax, stream())
        return
    from .graph import side_stream, _SIDE_PENDING
    side = side_stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    # the pass outlives the caller's references under no_grad (the autograd ctx that holds S /
    # den / argmax is dropped when apply returns): mark every buffer it touches as in use on the
    # side stream, so the caching allocator cannot hand one to the next layer's GEMM before the
    # pass has finished with it (LazyAlpha.materialize does the same)
    ei = graph._ei_flat if graph._ei_flat is not None else graph.source
    for t in (S, M_ord, den, argmax, alpha, ei, graph.rowptr, graph.perm, graph.meta):
        if t is not None:
            t.record_stream(side)
    with torch.cuda.stream(side):
        with _span("attention_alpha", (graph.edge_bound, sh.NH)):
            _attention_alpha(graph, S, M_ord, den, sh, alpha, argmax, stream())
    _SIDE_PENDING[dev] = True


def _attention_alpha(graph: Graph, S, M_ord, den, sh: "LayerShape", alpha, argmax, s):
    """alpha in edge_index' order (models/gat_layer.py:106-110): iterates edge_index' itself, so
    both its reads and the alpha writes are coalesced; |edge_index'| is read on the device."""
    ei_p, is64, ld = graph.ei_args
    call("gatx_attention_alpha_ei", ei_p, is64, ld, graph.edge_bound, graph.e2_ptr, ptr(S),
         ptr(M_ord), ptr(den), sh.NH, int(sh.const), ptr(graph.rowptr), ptr(graph.perm),
         ptr(alpha), ptr(argmax), s)


def edge_heads_per_item(sh: LayerShape) -> int:
    """Heads per edge work item: ~256+ floats of gathered row per item, so one XCD's L2 holds
    the sweep's slice of the rows (measured inside the PPI forward: 1 head of 256 per item beats
    2 and 4); the largest divisor of NH up to 8 (the batch phase keeps the item's heads in
    registers). Head-mean layers use the same rule: a head group smaller than NH runs as one
    launch per group, accumulating into the output in stream order (PPI L2: 6 heads x 124
    floats -> 3 groups of 2, each group's per-graph slice ~2.2 MB instead of 6.7 MB)."""
    hs = tuning.get("heads_per_item")
    if hs > 0 and sh.NH % hs == 0 and hs <= 8:
        return hs
    if not sh.concat:
        hm = tuning.get("mean_heads")
        if hm > 0 and sh.NH % hm == 0 and hm <= 8:
            return hm
        # measured at PPI L2 (6 x 124 floats), edge pass per step: groups of 6 / 3 / 2 / 1
        # heads 0.608 / 0.580 / 0.596 / 0.688 ms (the pass is bound by L2->CU gather bandwidth,
        # ~16 TB/s, more than by HBM): ~384 floats of row per group
        return max(d for d in range(1, 9) if sh.NH % d == 0 and d * sh.Fp <= max(384, sh.Fp))
    return max(d for d in range(1, 9) if sh.NH % d == 0 and d * sh.Fp <= max(256, sh.Fp))


def hub_args(graph: Graph, sh: LayerShape, hs: int, group_count: int, dev):
    """The trailing hub-splitting arguments of gatx_edge_forward_hubs: (hub_edges, hubs, count,
    bound, partials). Segments longer than tuning hub_edges (8192) edges are aggregated in pieces
    by parallel waves (degree skew). Engaged for graphs of more than
    tuning hub_min_edges (2^22) input edges: there the plan and the combine launch cost nothing
    next to the edge pass; a smaller graph's longest segment costs one wave at most 2^22 edges."""
    T = tuning.get("hub_edges")
    if T <= 0 or graph.num_input_edges <= tuning.get("hub_min_edges"):
        return (0, None, None, 0, None)
    hubs, count, bound = graph.hub_plan(T)
    nb = lib.gatx_edge_forward_hub_part_bytes(bound, sh.NH, sh.F, hs, group_count)
    part = torch.empty(max(nb, 4), dtype=torch.uint8, device=dev)
    return (T, ptr(hubs), ptr(count), bound, ptr(part))


def bwd_hub_args(graph: Graph, NH: int, F: int, dev, source: bool):
    """The trailing hub-splitting arguments of gatx_edge_backward_{dst,src}_hubs, over the
    destination CSR (source=False) or the transpose (source=True), for graphs past the forward's
    2^22-edge threshold. The backward's items are one head each (the forward's carry up to 8), so
    a segment costs one wave 8x less there: on R-MAT 1e7 / 1.6e8 splitting at 8192 edges gained
    nothing (dst pass 19.06 ms unsplit vs 17.84 + 1.18 split; profiles/r03m), so the backward
    splits only segments past tuning bwd_hub_edges = 65536 edges — the guard against extreme skew
    (a star graph's hub would otherwise be one wave's walk). tuning bwd_hubs=0: never split."""
    T = tuning.get("bwd_hub_edges")
    if (T <= 0 or tuning.get("bwd_hubs") == 0
            or graph.num_input_edges <= tuning.get("hub_min_edges")):
        return (0, None, None, 0, None)
    hubs, count, bound = graph.hub_plan(T, source)
    nb = lib.gatx_edge_backward_hub_part_bytes(bound, NH, F, int(source))
    part = torch.empty(max(nb, 4), dtype=torch.uint8, device=dev)
    return (T, ptr(hubs), ptr(count), bound, ptr(part))


def _edge_pass(rows, row_stride, S, M_ord, graph, sh, bias, p, seed, out, resid_p, elu, den,
               chunk, drop_args, dev, s):
    """The edge pass of a non-reassociated layer (concat, or head mean over head groups)."""
    N = graph.num_nodes
    hs = edge_heads_per_item(sh)
    ng = sh.NH // hs
    if sh.concat or ng == 1:
        hub = hub_args(graph, sh, hs, ng, dev)
        call("gatx_edge_forward_skip", ptr(rows), row_stride, sh.Fp, ptr(S), ptr(M_ord),
             ptr(graph.rowptr), ptr(graph.col), ptr(graph.perm), N, sh.NH, sh.F, hs,
             0, 0, 0, int(sh.concat), int(sh.const), ptr(bias), float(p), ptr(seed),
             ptr(out), sh.out_cols, resid_p, sh.out_cols, int(elu), ptr(den), chunk, *hub,
             *drop_args, None, s)
    else:   # head mean over groups: one launch per group, accumulated in stream order
        hub = hub_args(graph, sh, hs, 1, dev)
        for gi in range(ng):
            last = gi == ng - 1
            mode = 1 if gi == 0 else (3 if last else 2)
            call("gatx_edge_forward_skip", ptr(rows), row_stride, sh.Fp, ptr(S), ptr(M_ord),
                 ptr(graph.rowptr), ptr(graph.col), ptr(graph.perm), N, sh.NH, sh.F, hs,
                 gi, 1, mode, 0, int(sh.const), ptr(bias) if last else None, float(p),
                 ptr(seed), ptr(out), sh.out_cols, resid_p if last else None, sh.out_cols,
                 int(elu) if last else 0, ptr(den), chunk, *hub,
                 *(drop_args if last else (0.0, None)), None, s)


LDS_MAX_EDGES = 1 << 28   # edge_lds.hip: 32-bit record byte offsets
LDS_MAX_NODES = 1 << 25   # edge_lds.hip: records hold 64 src in an int32


def lds_blocks(graph: Graph, sh: LayerShape, side: bool = False, out_p: float = 0.0):
    """(segs, count, n_blocks) when this layer's edge pass takes the LDS-staged kernels
    (csrc/edge_lds.hip; tuning edge_lds, and edge_lds_mean for head-mean layers): a layer of <= 8
    heads on a graph whose node
    blocks (gatx_graph_segments) fit the LDS image; else None. side: a first build of the blocks
    runs on the side stream (the caller joins it before the LDS pass). Graphs past the kernels'
    index limits take the L2-gather pass: the records hold 64 src in an int32 (N < 2^25) and the
    walk addresses them by 32-bit byte offsets (E' < 2^28, gatx_edge_lds_forward's check; the
    head-mean walk all heads' records from one base: 8 NH E' < 2^32; and it fuses no output
    dropout)."""
    if (not tuning.get("edge_lds") or (not sh.concat and not tuning.get("edge_lds_mean"))
            or sh.NH > 8
            or graph.edge_bound < tuning.get("lds_min_edges")
            or graph.edge_bound >= LDS_MAX_EDGES or graph.num_nodes >= LDS_MAX_NODES
            or (not sh.concat and (8 * sh.NH * graph.edge_bound >= (1 << 32) or out_p > 0))):
        return None
    return graph.lds_blocks(lib.gatx_edge_lds_rows(), side)


def fold_scores_into_gemm(sh: LayerShape) -> bool:
    """Compute S as 2NH extra GEMM columns only when they fit the last column tile for free;
    otherwise (e.g. Dp = 1024: a whole extra 128-wide tile, +12% GEMM time) project Wh alone and
    derive S from it with gatx_node_scores (one extra read of Wh)."""
    if sh.H2 == 0:
        return True
    if 2 * sh.NH * sh.Dp * 4 > 64 * 1024:
        return True
    return -(-(sh.Dp + sh.H2) // 128) == -(-sh.Dp // 128)


def use_reassociation(sh: LayerShape) -> bool:
    """Aggregate x rows instead of Wh rows when x is much narrower (PPI layer 0: 50 vs 1024):
    out_h = (sum alpha~ x[src]) W_h^T == sum alpha~ (x[src] W_h^T)."""
    if tuning.get("reassoc") == 0:
        return False
    return sh.concat and 2 * _round4(sh.F_in) <= sh.Dp and reassoc_heads_per_item(sh) > 0


def reassoc_heads_per_item(sh: LayerShape) -> int:
    """Heads sharing one gathered x row in the reassociated edge pass: the largest divisor of NH
    up to 8 whose HS * round4(F_in) row fits the edge kernel's 2048-float item (0: none fits)."""
    Fin_p = _round4(sh.F_in)
    fits = [d for d in range(1, 9) if sh.NH % d == 0 and d * Fin_p <= 2048]
    return max(fits) if fits else 0


def fuses_output_dropout(num_heads, out_features, in_features, concat, const_attention=False):
    """Whether a layer of this shape can apply the NEXT layer's input dropout in its own epilogue
    (gatx_edge_forward_drop): every layer whose output comes from the edge pass, i.e. all but
    the reassociated first-layer dataflow (its output comes from the batched GEMM's epilogue)."""
    return not use_reassociation(LayerShape(num_heads, out_features, in_features, concat,
                                            const_attention))


class LazyAlpha:
    """alpha of a forward that nothing has asked for yet (an inference forward without
    return_attention_weights): the reference computes and stores it in every forward
    (`models/gat_layer.py:106-110`); here the pass that writes it (gatx_attention_alpha_ei) runs
    when `normalised_attention_coeffs` is first read, from the softmax state the forward left (the
    node scores S, the global max and the denominators, all kept alive by this object) — the
    same kernel on the same inputs, so the same values as an eager forward. Training forwards
    stay eager: the backward's max() gradient needs the argmax entries that pass records.

    Streams: the forward's stream is remembered; a read from another stream first makes that
    stream wait for the forward's (and marks the saved buffers as used there, so the caching
    allocator cannot hand them out before the pass has read them). The pass reads edge_index'
    — with add_self_loops=False that is the caller's own edge_index — so edge_index must not be
    modified in place before alpha has been read (the reference has no such window: it writes
    alpha inside the forward)."""

    __slots__ = ("graph", "S", "M_ord", "den", "sh", "argmax", "fwd_stream")

    def __init__(self, graph, S, M_ord, den, sh, argmax):
        self.graph, self.S, self.M_ord, self.den, self.sh, self.argmax = \
            graph, S, M_ord, den, sh, argmax
        self.fwd_stream = torch.cuda.current_stream(S.device)

    def materialize(self) -> torch.Tensor:
        cur = torch.cuda.current_stream(self.S.device)
        if cur != self.fwd_stream:
            cur.wait_stream(self.fwd_stream)
            ei = self.graph._ei_flat if self.graph._ei_flat is not None else self.graph.source
            for t in (self.S, self.M_ord, self.den, self.argmax, ei, self.graph.rowptr,
                      self.graph.perm, self.graph.meta):
                t.record_stream(cur)
        alpha = torch.empty((max(self.graph.edge_bound, 1), self.sh.NH), dtype=torch.float32,
                            device=self.S.device)
        with _span("attention_alpha", (self.graph.edge_bound, self.sh.NH)):
            _attention_alpha(self.graph, self.S, self.M_ord, self.den, self.sh, alpha,
                             self.argmax, stream())
        return alpha


def layer_forward(x, W, a, bias, graph: Graph, sh: LayerShape, p: float, seed: int,
                  resid=None, elu=False, skip_W=None, out_p=0.0, out_seed=None,
                  want_alpha=True):
    """Returns out (= elu?(layer(x) + resid) when fused), alpha (edge_index' order; a LazyAlpha
    when want_alpha is False) and the saved state for the backward. skip_W: GATModel's Linear skip folded into the projection GEMM (its
    rows appended to W_aug; the GEMM writes the skip output R as a third output range and the
    edge pass / output projection epilogue adds it): resid = x W_skip_eff^T without a launch.
    out_p / out_seed: the next layer's input dropout applied by this layer's edge-pass epilogue
    (fuses_output_dropout must hold); the returned out is then the dropped output."""
    N = x.size(0)
    dev = x.device
    s = stream()
    E2 = graph.edge_bound   # allocation bound; kernels read |edge_index'| on the device
    f32 = dict(dtype=torch.float32, device=dev)
    chunk = tuning.get("edge_chunk")
    out = torch.empty((N, sh.out_cols), **f32)
    alpha = torch.empty((max(E2, 1), sh.NH), **f32) if want_alpha else None
    den = torch.empty((N, sh.NH), **f32)
    # argmax[0] (tie count) is reset by gatx_attention_max; M_ord is written by it
    argmax = torch.empty(ARGMAX_CAP + 2, dtype=torch.int64, device=dev)
    M_ord = torch.empty(1, dtype=torch.int32, device=dev)
    C = sh.skip_cols
    R = torch.empty((N, C), **f32) if C else None   # the folded skip's output
    if R is not None:
        resid = R
    resid_p = ptr(resid) if resid is not None else None
    W_aug = augmented_weight(W, a, sh, skip_W)
    saved = dict(W_aug=W_aug, M_ord=M_ord, den=den, argmax=argmax, Wh=None, out_p=float(out_p),
                 out_seed=out_seed)
    drop_args = (float(out_p), ptr(out_seed) if out_p > 0 else None)
    if use_reassociation(sh):
        if out_p > 0:
            raise RuntimeError("gatx: output dropout is not fused into a reassociated layer")
        Fin_p = _round4(sh.F_in)
        if Fin_p != sh.F_in:
            x_rows = torch.empty((N, Fin_p), **f32)
            call("gatx_pad_rows", ptr(x), N, sh.F_in, sh.F_in, ptr(x_rows), Fin_p, s)
        else:
            x_rows = x
        S = torch.empty((N, max(sh.H2, 1)), **f32)
        if not sh.const or C:
            # S = x [A_src W; A_dst W]^T, and the folded skip's R = x W_skip_eff^T from the rows
            # after them as the second output range of the same launch
            with _span("gemm_scores", (N, sh.H2 + C, sh.F_in)):
                call("gatx_gemm_f32", N, sh.H2 + C, sh.F_in, ptr(x), sh.F_in, 1,
                     ptr(W_aug) + 4 * sh.Dp * sh.F_in, 1, sh.F_in, ptr(S), max(sh.H2, 1), sh.H2,
                     ptr(R) if C else None, max(C, 1), 0,
                     *gemm_workspace(N, sh.H2 + C, sh.F_in, dev), s)
        if not sh.const:
            with _span("attention_max", (E2, sh.NH)):
                call("gatx_attention_max", ptr(graph.col), ptr(graph.rowidx), E2, graph.e2_ptr,
                     ptr(S), sh.NH, ptr(M_ord), ptr(argmax), ptr(_max_ws(dev)), s)
        Z = torch.empty((N, sh.NH * Fin_p), **f32)
        with _span("edge_forward", (N, E2, sh.NH, Fin_p, "x")):
            hs_x = reassoc_heads_per_item(sh)   # heads sharing one x row
            hub = hub_args(graph, LayerShape(sh.NH, Fin_p, sh.F_in, True, sh.const), hs_x,
                           sh.NH // hs_x, dev)
            call("gatx_edge_forward_hubs", ptr(x_rows), Fin_p, 0, ptr(S), ptr(M_ord),
                 ptr(graph.rowptr), ptr(graph.col), ptr(graph.perm), N, sh.NH, Fin_p, hs_x,
                 0, 0, 0, 1,
                 int(sh.const), None, float(p), ptr(seed), ptr(Z), sh.NH * Fin_p, None, 0, 0,
                 ptr(den), chunk, *hub, s)
        if want_alpha:
            _alpha_pass(graph, S, M_ord, den, sh, alpha, argmax, dev)
        else:
            alpha = LazyAlpha(graph, S, M_ord, den, sh, argmax)
        Wp = padded_weight(W, Fin_p, sh.cache_weights)   # float4-readable rows
        saved["Wp"] = Wp   # the backward's batched GEMMs read the same padded copy
        with _span("gemm_out", (N, sh.F, sh.F_in, sh.NH)):
            call("gatx_gemm_f32_batched", sh.NH, N, sh.F, sh.F_in, ptr(Z), sh.NH * Fin_p, 1,
                 Fin_p, ptr(Wp), 1, Fin_p, sh.F * Fin_p, ptr(out), sh.NH * sh.F, sh.F, 0,
                 ptr(bias), sh.F, resid_p, sh.out_cols, sh.F, int(elu), s)
        saved.update(S=S, reassoc=True, Z=Z, x_rows=x_rows)
        return out, alpha, saved
    # node blocks of an LDS-staged layer: built on the side stream while the projection GEMM runs
    blocks = lds_blocks(graph, sh, side=True, out_p=out_p)
    Wh = torch.empty((N, sh.Dp), **f32)
    S = torch.empty((N, max(sh.H2, 1)), **f32)
    # the weight operand pre-split into fp16 planes (gemm_f16p.hip; None: in-loop split)
    planes = projection_planes(W_aug, sh, N)
    pp = ptr(planes) if planes is not None else None
    if C:   # one launch: [Wh | S | R] = x [W_aug; W_skip_eff]^T into three outputs
        with _span("gemm", (N, sh.K_aug + C, sh.F_in, sh.NH, sh.F)):
            call("gatx_gemm_planes", N, sh.K_aug + C, sh.F_in, ptr(x), sh.F_in, ptr(W_aug),
                 sh.F_in, pp, ptr(Wh), sh.Dp, sh.Dp, ptr(S), max(sh.H2, 1), sh.K_aug, ptr(R), C,
                 0, None, 0, 0, None, 0, None, *gemm_workspace(N, sh.K_aug + C, sh.F_in, dev), s)
    elif fold_scores_into_gemm(sh):
        with _span("gemm", (N, sh.K_aug, sh.F_in, sh.NH, sh.F)):
            call("gatx_gemm_planes", N, sh.K_aug, sh.F_in, ptr(x), sh.F_in, ptr(W_aug), sh.F_in,
                 pp, ptr(Wh), sh.Dp, sh.Dp, ptr(S), max(sh.H2, 1), -1, None, 0, 0, None, 0, 0,
                 None, 0, None, *gemm_workspace(N, sh.K_aug, sh.F_in, dev), s)
    elif tuning.get("fused_scores"):
        # S reduced from the projection's accumulators in its epilogue (no second read of Wh)
        with _span("gemm", (N, sh.Dp, sh.F_in, sh.NH, sh.F)):
            nb = lib.gatx_projection_scores_workspace_bytes(N, sh.Dp, sh.F_in, sh.NH)
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
            call("gatx_gemm_planes", N, sh.Dp, sh.F_in, ptr(x), sh.F_in, ptr(W_aug), sh.F_in, pp,
                 ptr(Wh), sh.Dp, sh.Dp, None, 0, -1, None, 0, 0, ptr(a), sh.NH, sh.F, ptr(S), 0,
                 None, ptr(ws), nb, s)
    else:   # (tuning fused_scores=0: the projection alone, then the score pass over Wh)
        with _span("gemm", (N, sh.Dp, sh.F_in, sh.NH, sh.F)):
            call("gatx_gemm_planes", N, sh.Dp, sh.F_in, ptr(x), sh.F_in, ptr(W_aug), sh.F_in, pp,
                 ptr(Wh), sh.Dp, sh.Dp, None, 0, -1, None, 0, 0, None, 0, 0, None, 0, None,
                 *gemm_workspace(N, sh.Dp, sh.F_in, dev), s)
        with _span("node_scores", (N, sh.NH, sh.F)):
            call("gatx_node_scores", ptr(Wh), N, sh.NH, sh.F, ptr(a), ptr(S), s)
    # the previous layer's side-stream alpha pass and this layer's node blocks ran under the GEMM
    join_side(dev)
    if not sh.const:
        with _span("attention_max", (E2, sh.NH)):
            call("gatx_attention_max", ptr(graph.col), ptr(graph.rowidx), E2, graph.e2_ptr,
                 ptr(S), sh.NH, ptr(M_ord), ptr(argmax), ptr(_max_ws(dev)), s)
    if blocks is not None:
        # LDS-staged edge pass (csrc/edge_lds.hip): records (den, alpha, ties, {4 src, alpha~}
        # per head and CSR slot), then one workgroup per (node block, head, 16-float chunk)
        segs, count, nblocks = blocks
        rec = torch.empty((sh.NH, max(E2, 1)), dtype=torch.int64, device=dev)
        with _span("edge_records", (E2, sh.NH)):
            call("gatx_edge_records", ptr(S), ptr(M_ord), ptr(graph.rowptr), ptr(graph.col),
                 ptr(graph.perm), N, E2, sh.NH, int(sh.const), float(p), ptr(seed), ptr(rec),
                 ptr(den), ptr(alpha) if want_alpha else None,
                 ptr(argmax) if want_alpha else None, s)
        with _span("edge_forward", (N, E2, sh.NH, sh.F, sh.concat, "lds")):
            call("gatx_edge_lds_forward" if sh.concat else "gatx_edge_lds_mean_forward",
                 ptr(Wh), sh.Dp, ptr(graph.rowptr), N, ptr(rec), E2,
                 ptr(segs), ptr(count), nblocks, sh.NH, sh.F, ptr(bias), ptr(out), sh.out_cols,
                 resid_p, sh.out_cols, int(elu), *drop_args, s)
        if not want_alpha:
            alpha = LazyAlpha(graph, S, M_ord, den, sh, argmax)
        saved.update(Wh=Wh, S=S, reassoc=False)
        return out, alpha, saved
    with _span("edge_forward", (N, E2, sh.NH, sh.F, sh.concat)):   # local + generic: one record
        _edge_pass(Wh, sh.Dp, S, M_ord, graph, sh, bias, p, seed, out, resid_p, elu, den, chunk,
                   drop_args, dev, s)
    if want_alpha:
        _alpha_pass(graph, S, M_ord, den, sh, alpha, argmax, dev)
    else:
        alpha = LazyAlpha(graph, S, M_ord, den, sh, argmax)
    saved.update(Wh=Wh, S=S, reassoc=False)
    return out, alpha, saved


def layer_backward(g_out, g_alpha, x, W, a, bias, graph: Graph, sh: LayerShape, p: float,
                   seed: int, saved, need_x: bool, need_W: bool, need_a: bool, need_bias: bool,
                   out=None, elu=False, need_resid=False, resid_is_x=False, need_skip=False):
    """Gradients of layer_forward; returns (g_x, g_W, g_a, g_bias, g_resid). With resid_is_x
    (GATModel's identity skip) the skip gradient is folded into g_x by the g_x GEMM's
    accumulate epilogue and g_resid is None. With a folded Linear skip (sh.skip_cols) its
    gradient rides in G_aug's last columns: g_x includes it, and with need_skip the gradient of
    W_skip_eff is left in saved["g_skip_eff"]."""
    N = x.size(0)
    dev = x.device
    s = stream()
    f32 = dict(dtype=torch.float32, device=dev)
    g_out = g_out.contiguous()
    E2 = graph.edge_bound   # g_raw row stride; kernels read |edge_index'| on the device
    graph.ensure_transpose()
    if saved.get("reassoc") and not need_x and not sh.const and sh.NH <= 8:
        return _reassoc_backward(g_out, g_alpha, x, W, a, bias, graph, sh, p, seed, saved,
                                 need_W, need_a, need_bias, out, elu, need_resid, need_skip)
    if saved["Wh"] is None:   # reassociated forward never built Wh: project now
        Wh = torch.empty((N, sh.Dp), **f32)
        call("gatx_gemm_f32", N, sh.Dp, sh.F_in, ptr(x), sh.F_in, 1, ptr(saved["W_aug"]), 1,
             sh.F_in, ptr(Wh), sh.Dp, sh.Dp, None, 0, 0, *gemm_workspace(N, sh.Dp, sh.F_in, dev),
             s)
        saved["Wh"] = Wh
    go = torch.empty((N, sh.Dp if sh.concat else sh.Fp), **f32)
    C = sh.skip_cols
    # folded skip: its gradient g_pre occupies G_aug's columns K_aug.. (written by prepare_go),
    # so the g_x and weight-gradient GEMMs below cover the skip in the same launches
    ldg = _round4(sh.K_aug + C) if C else sh.ldg
    G_aug = torch.empty((N, ldg), **f32)
    g_pre, pre_ld, pre_p = None, sh.out_cols, None
    if C:
        pre_ld, pre_p = ldg, ptr(G_aug) + 4 * sh.K_aug
    elif need_resid or (need_bias and elu):
        # concat with F % 4 == 0: go already is the gradient before the skip-add (same layout,
        # scale 1), and go is dead once the source pass has run, so it doubles as g_pre
        g_pre = go if (sh.concat and sh.F % 4 == 0) else torch.empty((N, sh.out_cols), **f32)
        pre_p = ptr(g_pre)
    out_p = saved.get("out_p", 0.0)
    # KernelTimer record info (bench.py prices each backward record from it)
    binfo = (N, E2, sh.F_in, sh.NH, sh.F, sh.concat, C, bool(elu), False)
    with _span("bwd_prepare_go", binfo):
        call("gatx_prepare_go_ex", ptr(g_out), ptr(out) if elu else None, N, sh.NH, sh.F,
             int(sh.concat), int(elu), ptr(go), pre_p, pre_ld, out_p,
             ptr(saved["out_seed"]) if out_p > 0 else None, s)
    g_raw = g_corr = None
    if not sh.const:
        g_raw = torch.empty((sh.NH, max(E2, 1)), **f32)
        gsd = torch.empty((N, sh.NH), **f32)
        with _span("bwd_edge_dst", binfo):
            call("gatx_edge_backward_dst_hubs", ptr(saved["Wh"]), sh.Dp, sh.Fp, ptr(saved["S"]),
             ptr(saved["M_ord"]), ptr(saved["den"]), ptr(graph.rowptr), ptr(graph.col),
                 ptr(graph.perm), N, E2, sh.NH, sh.F, ptr(go), sh.Dp if sh.concat else sh.Fp,
                 sh.Fp if sh.concat else 0, float(p), ptr(seed),
                 ptr(g_alpha.contiguous()) if g_alpha is not None else None, ptr(g_raw),
                 ptr(gsd), ptr(G_aug), ldg, sh.Dp, *bwd_hub_args(graph, sh.NH, sh.F, dev, False),
                 s)
    src_blocks = (lds_blocks(graph, sh) if sh.concat and sh.F % 4 == 0
                  and tuning.get("edge_lds_bwd") else None)
    if src_blocks is not None:
        # the source pass as the forward's LDS walk over the transposed CSR, go's rows staged
        # (csrc/edge_lds.hip: gatx_edge_records_src, then gatx_edge_lds_forward into G_aug)
        segs, count, nblocks = src_blocks
        trec = torch.empty((sh.NH, max(E2, 1)), dtype=torch.int64, device=dev)
        with _span("bwd_edge_src", binfo + ("lds",)):
            call("gatx_edge_records_src", ptr(saved["S"]), ptr(saved["M_ord"]),
                 ptr(saved["den"]), ptr(graph.srowptr), ptr(graph.scol), ptr(graph.seid),
                 ptr(graph.perm), N, E2, sh.NH, int(sh.const), float(p), ptr(seed),
                 ptr(g_raw) if g_raw is not None else None, ptr(G_aug), ldg, sh.Dp, ptr(trec), s)
            call("gatx_edge_lds_forward", ptr(go), sh.Dp, ptr(graph.srowptr), N, ptr(trec), E2,
                 ptr(segs), ptr(count), nblocks, sh.NH, sh.F, None, ptr(G_aug), ldg, None, 0, 0,
                 0.0, None, s)
    else:
        with _span("bwd_edge_src", binfo):
            call("gatx_edge_backward_src_hubs", ptr(saved["S"]), ptr(saved["M_ord"]),
                 ptr(saved["den"]), ptr(graph.srowptr), ptr(graph.scol), ptr(graph.seid),
                 ptr(graph.perm), N, E2, sh.NH, sh.F, int(sh.concat), int(sh.const), float(p),
                 ptr(seed), ptr(go), ptr(g_raw), None, ptr(G_aug), ldg,
                 *bwd_hub_args(graph, sh.NH, sh.F, dev, True), s)
    if not sh.const:   # max()'s share, added into both logit-gradient columns of G_aug
        mws = torch.empty(lib.gatx_max_backward_workspace_bytes(), dtype=torch.uint8, device=dev)
        with _span("bwd_max", binfo):
            call("gatx_max_backward", ptr(saved["argmax"]), ptr(gsd), ptr(saved["S"]),
                 ptr(saved["M_ord"]), ptr(graph.col), ptr(graph.rowidx), N, E2, graph.e2_ptr,
                 sh.NH, None, ptr(G_aug), ldg, sh.Dp, ptr(mws), s)
    g_x = g_W = g_a = g_bias = None
    W_aug = saved["W_aug"]
    KC = sh.K_aug + C   # GEMM depth / rows over [g_Wh | g_s | g_skip]
    if need_bias and bias is not None:   # before g_pre may become g_x's accumulator
        g_bias = torch.empty_like(bias)
        src_p, src_ld = (pre_p, pre_ld) if elu else (ptr(g_out), sh.out_cols)
        with _span("bwd_colsum", binfo):
            call("gatx_colsum", src_p, N, sh.out_cols, src_ld, ptr(g_bias), s)
    fold = resid_is_x and need_x and g_pre is not None
    # exact max |.| of G_aug's rows (the g_x GEMM's row scales) and columns (the weight-gradient
    # GEMM's), from ONE read of G_aug (gatx_absmax_rows_cols); computed on first use
    stats_box = []

    def g_aug_stats():
        if not stats_box:
            if KC > 2048:   # (the pass holds at most 2048 columns per lane set; the GEMMs then
                stats_box.append((None, None))   # scale rows by their first K-tile)
                return stats_box[0]
            rowmax = torch.empty(N, **f32)
            colmax = torch.empty(KC, **f32)
            with _span("bwd_gaug_stats", binfo):
                call("gatx_absmax_rows_cols", ptr(G_aug), N, KC, ldg, ptr(rowmax), ptr(colmax), s)
            stats_box.append((rowmax, colmax))
        return stats_box[0]
    if need_x:
        g_x = g_pre if fold else torch.empty((N, sh.F_in), **f32)
        big = N * sh.F_in * KC >= (1 << 27)
        with_planes = big and use_weight_planes(sh.F_in, KC, N)
        # (G_aug's row maxima before the span: the statistics pass has its own)
        stats = g_aug_stats() if with_planes else None
        with _span("bwd_gemm_gx", binfo + (bool(fold),)):
            if big:
                # W_aug^T (F_in x K_aug, 4 MB at PPI): both GEMM operands k-contiguous (the
                # n-contiguous B staging of W_aug as stored ran this product ~25% slower), and
                # pre-split into fp16 planes for the f16x3 kernel (gemm_f16p.hip)
                W_augT = torch.empty((sh.F_in, ldg), **f32)
                call("gatx_transpose_f32", KC, sh.F_in, ptr(W_aug), sh.F_in, ptr(W_augT), ldg, s)
                planes_t = None
                if with_planes:
                    planes_t = build_weight_planes(W_augT, sh.F_in, KC, ldg)
                call("gatx_gemm_planes", N, sh.F_in, KC, ptr(G_aug), ldg, ptr(W_augT), ldg,
                     ptr(planes_t) if planes_t is not None else None, ptr(g_x), sh.F_in,
                     sh.F_in, None, 0, -1, None, 0, int(fold), None, 0, 0, None, 1,
                     ptr(stats[0]) if planes_t is not None and stats[0] is not None else None,
                     *gemm_workspace(N, sh.F_in, KC, dev), s)
            else:   # small layers are launch-bound: read W_aug as stored (no transpose launch)
                call("gatx_gemm_f32", N, sh.F_in, KC, ptr(G_aug), ldg, 1, ptr(W_aug), sh.F_in,
                     1, ptr(g_x), sh.F_in, sh.F_in, None, 0, int(fold),
                     *gemm_workspace(N, sh.F_in, KC, dev), s)
    if need_W or need_a or need_skip:
        gW_aug = torch.empty((KC, sh.F_in), **f32)
        ws_bytes = lib.gatx_gemm_splitk_workspace_bytes(KC, sh.F_in, N)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        # the f16x3 weight-gradient kernel needs G_aug's exact column maxima
        colmax = g_aug_stats()[1] if use_wgrad_f16(KC, sh.F_in, N) else None
        with _span("bwd_gemm_gw", binfo):
            if colmax is not None:
                call("gatx_gemm_wgrad", KC, sh.F_in, N, ptr(G_aug), ldg, ptr(x), sh.F_in,
                     ptr(colmax), ptr(gW_aug), sh.F_in, ptr(ws), ws_bytes, s)
            else:
                call("gatx_gemm_f32_splitk", KC, sh.F_in, N, ptr(G_aug), 1, ldg, ptr(x),
                     sh.F_in, 1, ptr(gW_aug), sh.F_in, 0, ptr(ws), ws_bytes, s)
        g_W = torch.empty_like(W)
        g_a = torch.empty_like(a) if a is not None else None
        with _span("bwd_weight_grads", binfo):
            call("gatx_weight_grads", ptr(gW_aug), ptr(W), ptr(a), sh.NH, sh.F, sh.F_in,
                 ptr(g_W), ptr(g_a), s)
        if need_skip:
            saved["g_skip_eff"] = gW_aug[sh.K_aug:]
    g_resid = None
    if need_resid and not fold:
        g_resid = g_pre
    return (g_x, (g_W if need_W else None), (g_a if need_a else None), g_bias, g_resid)


# _reassoc_backward: smallest N * C whose skip-gradient copy costs more than one more launch
SKIP_FROM_GO_MIN = 1 << 22


def _reassoc_backward(g_out, g_alpha, x, W, a, bias, graph: Graph, sh: LayerShape, p, seed,
                      saved, need_W, need_a, need_bias, out, elu, need_resid, need_skip=False):
    """Backward of the reassociated first layer when its input needs no gradient (the model
    input): never forms Wh or its (N, NH*F) gradient.
      g_Z[n,h] = go[n,h] . W_h                      batched GEMM (g_Z[n,h] . x_src == g_alpha)
      dst pass over x rows (F_in floats, not NH*F)  -> g_raw', g_s_dst
      src scores: g_s_src = sum over out-edges      (no row gathers)
      g_W_h = go_h^T Z_h                            batched split-K GEMM, Z saved by the forward
      g_W_score = [g_s_src | g_s_dst]^T x           split-K GEMM
    then gatx_weight_grads maps g_W_aug to (g_W, g_a) exactly as the general path."""
    N = x.size(0)
    dev = x.device
    s = stream()
    f32 = dict(dtype=torch.float32, device=dev)
    E2 = graph.edge_bound
    NH, F, Fp, F_in = sh.NH, sh.F, sh.Fp, sh.F_in
    Fin_p = _round4(F_in)
    Z, x_rows = saved["Z"], saved["x_rows"]
    go = torch.empty((N, sh.Dp), **f32)
    C = sh.skip_cols
    # [g_s_src | g_s_dst | g_skip]: a folded skip's gradient in G_s's last columns, so the score
    # rows' split-K GEMM also yields the skip weight's gradient. When go already holds it (F % 4
    # == 0: go's head-padded rows ARE the skip output's layout, C = NH F = Dp) the skip rows'
    # GEMM reads go itself instead: no 4 N C-byte copy (184 MB at the all-skip PPI variant's L0
    # over 20 graphs) for one more launch, so only where the copy outweighs a launch
    skip_from_go = bool(C) and C == sh.Dp and F % 4 == 0 and N * C >= SKIP_FROM_GO_MIN
    lds = _round4(2 * NH + C) if (C and not skip_from_go) else 2 * NH
    G_s = torch.empty((N, lds), **f32)
    g_pre, pre_ld, pre_p = None, sh.out_cols, None
    if C and not skip_from_go:
        pre_ld, pre_p = lds, ptr(G_s) + 4 * 2 * NH
    elif C:
        pass
    elif need_resid or (need_bias and elu):
        g_pre = torch.empty((N, sh.out_cols), **f32)
        pre_p = ptr(g_pre)
    binfo = (N, E2, F_in, NH, F, True, C, bool(elu), True)
    with _span("bwd_prepare_go", binfo):
        call("gatx_prepare_go_ex", ptr(g_out), ptr(out) if elu else None, N, NH, F, 1,
             int(elu), ptr(go), pre_p, pre_ld, 0.0, None, s)
    Wp = saved.get("Wp")    # [NH*F][Fin_p], zero tail: the forward's copy
    if Wp is None:
        Wp = padded_weight(W, Fin_p, sh.cache_weights)
    g_Z = torch.empty((N, NH * Fin_p), **f32)
    with _span("bwd_gemm_gz", binfo):
        call("gatx_gemm_f32_batched", NH, N, Fin_p, F, ptr(go), sh.Dp, 1, Fp, ptr(Wp), Fin_p, 1,
             F * Fin_p, ptr(g_Z), NH * Fin_p, Fin_p, 0, None, 0, None, 0, 0, 0, s)
    g_raw = torch.empty((NH, max(E2, 1)), **f32)
    gsd = torch.empty((N, NH), **f32)
    with _span("bwd_edge_dst", binfo):
        call("gatx_edge_backward_dst_hubs", ptr(x_rows), Fin_p, 0, ptr(saved["S"]),
             ptr(saved["M_ord"]), ptr(saved["den"]), ptr(graph.rowptr), ptr(graph.col),
             ptr(graph.perm), N, E2, NH, Fin_p, ptr(g_Z), NH * Fin_p, Fin_p, float(p), ptr(seed),
             ptr(g_alpha.contiguous()) if g_alpha is not None else None, ptr(g_raw), ptr(gsd),
             ptr(G_s), lds, 0, *bwd_hub_args(graph, NH, Fin_p, dev, False), s)
    with _span("bwd_src_scores", binfo):
        call("gatx_edge_backward_src_scores", ptr(graph.srowptr), ptr(graph.seid), N, E2, NH,
             ptr(g_raw), None, ptr(G_s), lds, 0, s)
    mws = torch.empty(lib.gatx_max_backward_workspace_bytes(), dtype=torch.uint8, device=dev)
    with _span("bwd_max", binfo):
        call("gatx_max_backward", ptr(saved["argmax"]), ptr(gsd), ptr(saved["S"]),
             ptr(saved["M_ord"]), ptr(graph.col), ptr(graph.rowidx), N, E2, graph.e2_ptr, NH,
             None, ptr(G_s), lds, 0, ptr(mws), s)
    g_W = g_a = g_bias = None
    if need_W or need_a or need_skip:
        gW_aug = torch.empty((sh.K_aug + C, F_in), **f32)
        # main rows, head h at rows h*Fp.. : go_h^T (F x N) . Z_h (N x F_in)
        wb = lib.gatx_gemm_splitk_batched_workspace_bytes(NH, F, F_in, N)
        ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
        with _span("bwd_gemm_gw_z", binfo):
            call("gatx_gemm_f32_splitk_batched", NH, F, F_in, N, ptr(go), 1, sh.Dp, Fp, ptr(Z),
                 NH * Fin_p, 1, Fin_p, ptr(gW_aug), F_in, Fp * F_in, 0, ptr(ws), wb, s)
        # score rows (+ folded skip rows): G_s^T (2NH + C x N) . x (N x F_in)
        rows_s = 2 * NH if skip_from_go else 2 * NH + C
        wb2 = lib.gatx_gemm_splitk_workspace_bytes(rows_s, F_in, N)
        ws2 = torch.empty(max(wb2, 1), dtype=torch.uint8, device=dev)
        with _span("bwd_gemm_gs", binfo):
            call("gatx_gemm_f32_splitk", rows_s, F_in, N, ptr(G_s), 1, lds, ptr(x), F_in, 1,
                 ptr(gW_aug) + 4 * sh.Dp * F_in, F_in, 0, ptr(ws2), wb2, s)
        if skip_from_go:   # the skip rows: go^T (C x N) . x (N x F_in)
            wb3 = lib.gatx_gemm_splitk_workspace_bytes(C, F_in, N)
            ws3 = torch.empty(max(wb3, 1), dtype=torch.uint8, device=dev)
            with _span("bwd_gemm_gs", binfo):
                call("gatx_gemm_f32_splitk", C, F_in, N, ptr(go), 1, sh.Dp, ptr(x), F_in, 1,
                     ptr(gW_aug) + 4 * sh.K_aug * F_in, F_in, 0, ptr(ws3), wb3, s)
        g_W = torch.empty_like(W)
        g_a = torch.empty_like(a)
        with _span("bwd_weight_grads", binfo):
            call("gatx_weight_grads", ptr(gW_aug), ptr(W), ptr(a), NH, F, F_in, ptr(g_W),
                 ptr(g_a), s)
        if need_skip:
            saved["g_skip_eff"] = gW_aug[sh.K_aug:]
    if need_bias and bias is not None:
        g_bias = torch.empty_like(bias)
        src_p, src_ld = (pre_p, pre_ld) if elu else (ptr(g_out), sh.out_cols)
        if elu and pre_p is None:   # (skip_from_go: go is the gradient before ELU, same layout)
            src_p, src_ld = ptr(go), sh.Dp
        with _span("bwd_colsum", binfo):
            call("gatx_colsum", src_p, N, sh.out_cols, src_ld, ptr(g_bias), s)
    return (None, (g_W if need_W else None), (g_a if need_a else None), g_bias,
            g_pre if need_resid else None)


class GATLayerFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, a, bias, resid, skip_W, graph, sh, p, seed, elu, out_p, out_seed):
        out, alpha, saved = layer_forward(x, W, a, bias, graph, sh, p, seed, resid, elu, skip_W,
                                          out_p, out_seed)
        ctx.graph, ctx.sh, ctx.p, ctx.seed, ctx.saved, ctx.elu = graph, sh, p, seed, saved, elu
        ctx.has_resid = resid is not None
        ctx.resid_is_x = resid is not None and resid is x
        ctx.has_skip = skip_W is not None
        ctx.save_for_backward(x, W, a, bias, out if elu else None, skip_W)
        # an unused output (alpha, when only out feeds the loss) arrives as None in backward
        # instead of a materialised (E', NH) zero tensor: no fill launch, no zero reads
        ctx.set_materialize_grads(False)
        return out, alpha

    @staticmethod
    def backward(ctx, g_out, g_alpha):
        x, W, a, bias, out, skip_W = ctx.saved_tensors
        if g_out is None:
            g_out = torch.zeros((x.size(0), ctx.sh.out_cols), dtype=torch.float32,
                                device=x.device)
        nx, nW, na, nb, nr, ns = ctx.needs_input_grad[:6]
        sh = ctx.sh
        g_x, g_W, g_a, g_b, g_r = layer_backward(
            g_out, g_alpha, x, W, a, bias, ctx.graph, sh, ctx.p, ctx.seed, ctx.saved, nx, nW,
            na, nb, out=out, elu=ctx.elu, need_resid=bool(ctx.has_resid and nr),
            resid_is_x=ctx.resid_is_x, need_skip=bool(ctx.has_skip and ns))
        g_s = None
        if ctx.has_skip and ns:
            # gradient of W_skip_eff: W_skip's own for concat / one head; a head-mean layer's
            # W_skip gets it in every head block, / NH
            eff = ctx.saved.pop("g_skip_eff")
            if sh.concat or sh.NH == 1:
                g_s = eff
            else:
                g_s = torch.empty_like(skip_W)
                call("gatx_skip_weight_grad", ptr(eff), sh.NH, sh.skip_cols, sh.F_in, ptr(g_s),
                     stream())
        return g_x, g_W, g_a, g_b, g_r, g_s, None, None, None, None, None, None, None


class SkipProjectionFunction(torch.autograd.Function):
    """GATModel's Linear skip (`models/GATModel.py:107-110`, applied at `:136-145`) on the gatx
    GEMMs instead of a vendor BLAS call: out = x W^T for a concat layer, and for a head-mean
    layer the head mean of the projection as ONE product with the head-mean weight,
    mean_h(x W_h^T) = x (mean_h W_h)^T (F output columns instead of NH*F plus a mean reduction).
    Backward: g_x = g W_eff, g_W_eff = g^T x (deterministic split-K), g_W = g_W_eff broadcast
    over the heads / NH for the mean."""

    @staticmethod
    def forward(ctx, x, W, num_heads, out_features, mean):
        _require(x, "x")
        _require(W, "skip weight")
        x = x.contiguous()
        N, F_in = x.shape
        dev = x.device
        W_eff = (W.detach().view(num_heads, out_features, F_in).mean(0) if mean
                 else W.detach()).contiguous()
        cols = W_eff.size(0)
        out = torch.empty((N, cols), dtype=torch.float32, device=dev)
        with _span("skip", (N, cols, F_in)):
            call("gatx_gemm_f32", N, cols, F_in, ptr(x), F_in, 1, ptr(W_eff), 1, F_in, ptr(out),
                 cols, cols, None, 0, 0, *gemm_workspace(N, cols, F_in, dev), stream())
        ctx.save_for_backward(x, W_eff)
        ctx.num_heads, ctx.mean = num_heads, mean
        return out

    @staticmethod
    def backward(ctx, g):
        x, W_eff = ctx.saved_tensors
        N, F_in = x.shape
        cols = W_eff.size(0)
        dev = x.device
        s = stream()
        g = g.contiguous()
        g_x = g_W = None
        if ctx.needs_input_grad[0]:
            g_x = torch.empty((N, F_in), dtype=torch.float32, device=dev)
            call("gatx_gemm_f32", N, F_in, cols, ptr(g), cols, 1, ptr(W_eff), F_in, 1, ptr(g_x),
                 F_in, F_in, None, 0, 0, *gemm_workspace(N, F_in, cols, dev), s)
        if ctx.needs_input_grad[1]:
            gW = torch.empty((cols, F_in), dtype=torch.float32, device=dev)
            wb = lib.gatx_gemm_splitk_workspace_bytes(cols, F_in, N)
            ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
            call("gatx_gemm_f32_splitk", cols, F_in, N, ptr(g), 1, cols, ptr(x), F_in, 1,
                 ptr(gW), F_in, 0, ptr(ws), wb, s)
            g_W = gW.repeat(ctx.num_heads, 1).div_(ctx.num_heads) if ctx.mean else gW
        return g_x, g_W, None, None, None


class InputDropoutFunction(torch.autograd.Function):
    """GATModel's input dropout (`models/GATModel.py:130`, F.dropout) on gatx_dropout: the
    counter-based keep mask of the element index under a device seed (torch's generator draws
    the seed, so it follows torch.cuda.manual_seed and is graph-capturable); the backward is the
    same mask on the gradient. Used where the dropout cannot ride on the producing layer's
    epilogue (the model input, or after a reassociated layer)."""

    @staticmethod
    def forward(ctx, x, p, seed):
        _require(x, "x")
        x = x.contiguous()
        y = torch.empty_like(x)
        call("gatx_dropout", ptr(x), x.numel(), float(p), ptr(seed), ptr(y), stream())
        ctx.p, ctx.seed = float(p), seed
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        gx = torch.empty_like(g)
        call("gatx_dropout", ptr(g), g.numel(), ctx.p, ptr(ctx.seed), ptr(gx), stream())
        return gx, None, None


def input_dropout(x, p: float, seed):
    """y = dropout(x) with gatx's mask (see InputDropoutFunction); seed: int or device int64."""
    return InputDropoutFunction.apply(x, float(p), device_seed(seed, x.device))


def device_seed(seed, dev) -> torch.Tensor:
    """The dropout seed as the device scalar the kernels read: an int (tests, reproducible runs)
    is uploaded; a device int64 tensor (GATLayer draws one from torch's generator, so captured
    graphs get a fresh one per replay) is used as is."""
    if isinstance(seed, torch.Tensor):
        if seed.device != dev or seed.dtype != torch.int64 or seed.numel() != 1:
            raise RuntimeError("gatx: dropout seed must be one int64 on the layer's device")
        return seed.reshape(1)
    return torch.tensor([int(seed) & ((1 << 63) - 1)], dtype=torch.int64, device=dev)


def gat_layer(x, edge_index, W, a, bias, num_heads, out_features, concat, add_self_loops,
              const_attention=False, dropout_p=0.0, seed=0, graph: Graph | None = None,
              resid=None, elu=False, skip_weight=None):
    """Functional form of GATLayer.forward: returns (out, edge_index', alpha), the last two at
    their exact size (reads |edge_index'| from the device: one sync per new graph)."""
    out, graph, alpha = gat_layer_lazy(x, edge_index, W, a, bias, num_heads, out_features, concat,
                                       add_self_loops, const_attention, dropout_p, seed, graph,
                                       resid, elu, skip_weight)
    return out, graph.edge_index, alpha[:graph.num_edges]


def prepare_layer(x, edge_index, W, a, bias, num_heads, out_features, concat, add_self_loops,
                  const_attention=False, graph: Graph | None = None, resid=None,
                  skip_weight=None):
    """Argument checks of GATLayer.forward (the reference's own errors) and the layer's Graph:
    returns (x, W, a, resid, LayerShape, Graph) with contiguous tensors."""
    from .graph import graph_cache
    _require(x, "x")
    _require(W, "W")
    if a is not None:
        _require(a, "a")
    if bias is not None:
        _require(bias, "bias")
    if x.dim() != 2:
        raise RuntimeError(f"x must be (N, in_features), got {tuple(x.shape)}")
    x = x.contiguous()
    W = W.contiguous()
    a = a.contiguous() if a is not None else None
    sh = LayerShape(num_heads, out_features, x.size(1), concat, const_attention)
    sh.cache_weights = _cacheable(W, a, skip_weight)
    if skip_weight is not None:
        _require(skip_weight, "skip_weight")
        if resid is not None:
            raise RuntimeError("gatx: resid and skip_weight are exclusive")
        if tuple(skip_weight.shape) != (num_heads * out_features, x.size(1)):
            raise RuntimeError(f"skip weight shape {tuple(skip_weight.shape)} does not match "
                               f"({num_heads * out_features}, {x.size(1)})")
        sh.skip_cols = sh.out_cols
    if W.shape != (num_heads * out_features, x.size(1)):
        raise RuntimeError(f"W.weight shape {tuple(W.shape)} does not match "
                           f"({num_heads * out_features}, {x.size(1)})")
    if graph is None:
        graph = graph_cache.get(edge_index, x.size(0), add_self_loops)
    # E' == 0 iff E == 0 (with the rewrite an empty edge_index already raised in Graph)
    if graph.num_input_edges == 0 and not const_attention:
        # attention_weights.max() of an empty tensor (models/gat_layer.py:85)
        raise RuntimeError("max(): Expected reduction dim to be specified for input.numel() == 0.")
    if bias is not None and not concat and num_heads != 1:
        # output (N, F) += bias_param (NH*F,) cannot broadcast (models/gat_layer.py:134-135)
        raise RuntimeError(f"The size of tensor a ({out_features}) must match the size of tensor "
                           f"b ({num_heads * out_features}) at non-singleton dimension 1")
    if resid is not None:
        _require(resid, "resid")
        resid = resid.contiguous()
        if resid.shape != (x.size(0), sh.out_cols):
            raise RuntimeError(f"resid shape {tuple(resid.shape)} != {(x.size(0), sh.out_cols)}")
    return x, W, a, resid, sh, graph


def gat_layer_lazy(x, edge_index, W, a, bias, num_heads, out_features, concat, add_self_loops,
                   const_attention=False, dropout_p=0.0, seed=0, graph: Graph | None = None,
                   resid=None, elu=False, skip_weight=None, out_dropout=None,
                   defer_alpha=False):
    """gat_layer without any host sync: returns (out, graph, alpha_bound) where alpha_bound is
    (graph.edge_bound, NH) and its first graph.num_edges rows are alpha in edge_index' order.
    defer_alpha: with autograd off, alpha_bound is a LazyAlpha (its pass runs when it is read).
    resid / elu fuse GATModel's skip-add and ELU into the layer's epilogue:
    out = elu?(layer(x) + resid). skip_weight (GATModel's Linear skip, (NH*F, F_in)) folds the
    skip projection itself into the layer: resid = x W_skip^T (concat) or its head mean, computed
    by the layer's own projection GEMM. out_dropout = (p, device int64 seed): the next layer's
    input dropout (GATModel.py:130) applied by this layer's epilogue (see fuses_output_dropout);
    out is then the dropped output, with the mask of gatx_dropout under that seed."""
    x, W, a, resid, sh, graph = prepare_layer(x, edge_index, W, a, bias, num_heads, out_features,
                                              concat, add_self_loops, const_attention, graph,
                                              resid, skip_weight)
    if skip_weight is not None:
        skip_weight = skip_weight.contiguous()
    p = float(dropout_p)
    seed_t = device_seed(seed, x.device) if p > 0 else None
    out_p, out_seed = 0.0, None
    if out_dropout is not None and float(out_dropout[0]) > 0:
        out_p = float(out_dropout[0])
        out_seed = device_seed(out_dropout[1], x.device)
        if not fuses_output_dropout(num_heads, out_features, x.size(1), concat, const_attention):
            raise RuntimeError("gatx: out_dropout needs a layer whose output comes from the edge "
                               "pass (fuses_output_dropout)")
    if defer_alpha and not torch.is_grad_enabled():
        out, alpha, _ = layer_forward(x, W, a, bias, graph, sh, p, seed_t, resid, bool(elu),
                                      skip_weight, out_p, out_seed, want_alpha=False)
        return out, graph, alpha
    out, alpha = GATLayerFunction.apply(x, W, a, bias, resid, skip_weight, graph, sh, p, seed_t,
                                        bool(elu), out_p, out_seed)
    return out, graph, alpha


def _dst_row(graph):
    """(pointer, is64) of edge_index'[1] with unit stride."""
    ei = graph.edge_index
    if ei.stride(1) != 1:   # stream-ordered: the temporary outlives the enqueued kernel's use
        ei = ei.contiguous()
    return ptr(ei[1]), int(ei.dtype == torch.int64)


class AttentionNormFunction(torch.autograd.Function):
    """mean over layers of ||alpha_l * deg[dst] - 1||_1 / E' (`models/GATModel.py:189-234`) on
    gatx_attention_norm: one fused pass per layer over the CSR, gradient by
    gatx_attention_norm_backward."""

    @staticmethod
    def forward(ctx, graph, *alphas):
        E2 = graph.num_edges
        L = len(alphas)
        dev = alphas[0].device
        out = torch.empty(1, dtype=torch.float32, device=dev)
        ws = torch.empty(lib.gatx_attention_norm_workspace_bytes(), dtype=torch.uint8, device=dev)
        scale = 1.0 / (E2 * L) if E2 else float("nan")
        s = stream()
        alphas = tuple(a.contiguous() for a in alphas)
        for i, a in enumerate(alphas):
            _require(a, "attention")
            if a.dim() != 2 or a.size(0) != E2:
                raise RuntimeError(f"attention {i} has shape {tuple(a.shape)}, edge_index has "
                                   f"{E2} edges")
        if L <= 8:   # one pass over edge_index' for all layers (same bits as one per layer)
            ptrs = (ctypes.c_void_p * L)(*[ptr(a) for a in alphas])
            nhs = (ctypes.c_int * L)(*[a.size(1) for a in alphas])
            wsm = torch.empty(lib.gatx_attention_norm_multi_workspace_bytes(L), dtype=torch.uint8,
                              device=dev)
            with _span("attn_norm", (graph.num_nodes, E2, sum(a.size(1) for a in alphas))):
                call("gatx_attention_norm_multi", ctypes.addressof(ptrs), ctypes.addressof(nhs), L,
                     E2, *_dst_row(graph), ptr(graph.rowptr), scale, ptr(out), ptr(wsm), s)
        else:
            for i, a in enumerate(alphas):
                with _span("attn_norm", (graph.num_nodes, E2, a.size(1))):
                    call("gatx_attention_norm", ptr(a), E2, a.size(1), *_dst_row(graph),
                         ptr(graph.rowptr), scale, int(i > 0), ptr(out), ptr(ws), s)
        ctx.graph, ctx.scale = graph, scale
        ctx.save_for_backward(*alphas)
        return out.view(())

    @staticmethod
    def backward(ctx, g):
        graph = ctx.graph
        E2 = graph.num_edges
        g = g.to(torch.float32).contiguous().view(1)
        grads = []
        for a in ctx.saved_tensors:
            ga = torch.empty_like(a)
            with _span("attn_norm_bwd", (graph.num_nodes, E2, a.size(1))):
                call("gatx_attention_norm_backward", ptr(a), E2, a.size(1), *_dst_row(graph),
                     ptr(graph.rowptr), ptr(g), ctx.scale, ptr(ga), stream())
            grads.append(ga)
        return (None, *grads)


def attention_norm(edge_index, attention_list):
    """Functional GATModel.calc_attention_norm on the device (edge_index: the layers'
    edge_index', attention_list: their alphas)."""
    from .graph import graph_cache
    if not attention_list:
        raise RuntimeError("attention_norm: empty attention list")
    graph = graph_cache.for_edges(edge_index)
    return AttentionNormFunction.apply(graph, *attention_list)
