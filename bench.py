"""Benchmark: GAT-layer edges/s + achieved HBM GB/s, PPI 3-layer forward (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--graphs G] [--mode fwd|train]
                    [--workload ppi|pattern|rmat|cora|citeseer|pubmed]
                    [--wiring gatx|reference]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

`bench.py --gpus N` with N > 1 started as a single process starts the N ranks itself (children
under torch.distributed.run, before any GPU call here) and relays rank 0's line; under
torch.distributed.run (WORLD_SIZE set) each process is one rank and WORLD_SIZE must equal N.

Workload: per rank a synthetic PPI-shaped batch of G graphs (2245 nodes and 61318
uniformly random directed edges per graph; x ~ N(0,1), 50 features), the reference PPI config
(`run_config.py:18-33`: 3 layers, 4/4/6 heads, 256/256/121 features, concat/concat/mean, skip on
layer 1, ELU between layers) with random (xavier) weights, eval mode. One step = graph
preprocessing of a fresh batch (self-loop rewrite + CSR build, as every reference forward does
per layer) + the 3-layer forward. Weak scaling: each rank processes its own G graphs; the forward
has no exchange step, so there is no collective in the timed region (--mode train adds the
backward and the overlapped RCCL gradient all-reduce, gatx.distributed.GradientAllReducer).

value = (sum over ranks of layers x E' edges per step) / step time (max over ranks).
Byte accounting (all per step, all reported):
  unique_GBps        - the dataflow actually run, every array read/written once (gathered rows
                       once per node while the gathered matrix fits the 256 MB MALL, once per
                       edge beyond it): the HBM-compulsory traffic / step time
  roofline_time_frac - sum over kernels of max(unique bytes / 8 TB/s, flops / GEMM peak) over the
                       step time (<= 1 by construction when the clock is honest)
  hbm_measured       - rocprofv3 PMC bytes (FETCH_SIZE x 2 + WRITE_SIZE) per step from the
                       committed profiles/pmc_*.json summary, over this run's step time
  l2_gather_GBps     - SURVEY.md §8d's formula (one Wh row per EDGE, no reuse credited): the
                       gather rate the caches serve, NOT an HBM figure
roofline = the dominant kernel's flops (GEMM) or compulsory bytes (edge pass) per launch / its
average launch time, measured with HIP events on the launch stream over the last steps // 10
steps of the timed region (only those carry events: each record costs the stream ~10 us).
cpu_baseline = the reference dataflow restated in torch eager (oracle/torch_dataflow.py) on a
bounded sample, every available host core, rank 0, N=1 (the reference itself is timed in the
build container: bench/cpu_reference_baseline.json).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gat-pytorch_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
MALL_BYTES = 256 << 20       # Infinity Cache (MALL) capacity: the last on-chip level before HBM
FP32_MFMA_PEAK_TFS = 157.3   # v_mfma_f32_32x32x2_f32 dense peak (same table)
BF16_MFMA_PEAK_TFS = 2500.0  # dense bf16 MFMA peak (same table; no sparsity)
X3_PRODUCTS = 6              # bf16 MFMA products per fp32 multiply-add in the x3 split GEMM
F16X3_PRODUCTS = 3           # fp16 MFMA products per fp32 multiply-add in the f16x3 split GEMM


def gemm_roof():
    """Peak and kernel name of the projection GEMM in the library's active arithmetic mode.

    "f32": v_mfma_f32_32x32x2_f32, priced at the fp32 MFMA peak. "x3": each fp32 operand is
    split into three bf16 planes and every fp32 multiply-add costs six bf16 MFMA products
    (csrc/gemm_x3.hip), so the ceiling for fp32 flops is the dense bf16 peak / 6. "f16x3"
    (default): two fp16 planes per operand, three fp16 MFMA products per fp32 multiply-add
    (same kernel family, in-kernel x3 fallback for out-of-range tiles): dense fp16 peak (= bf16,
    2500 TF) / 3. Every mode's flops are fp32 GEMM flops of the same product.
    """
    from gatx import _lib
    mode = _lib.lib.gatx_get_gemm_mode()
    if mode == 2:
        from gatx import tuning
        f16p = tuning.get("f16p") != 0
        return dict(mode="f16x3", peak=BF16_MFMA_PEAK_TFS / F16X3_PRODUCTS,
                    prefix=("gemm_f16p_kernel<16, 0", "gemm_f16p_kernel<32, 0",
                            "gemm_x3_kernel<true, true, true, 0,"),
                    kernel=("gemm_f16p_kernel (weight as pre-split fp16 planes)" if f16p
                            else "gemm_x3_kernel") +
                           ", f16x3 arithmetic (fp32 as 2 fp16 planes x 3 MFMA products; peak = "
                           "dense fp16 2500 TF / 3)")
    if mode == 1:
        return dict(mode="x3", peak=BF16_MFMA_PEAK_TFS / X3_PRODUCTS, prefix="gemm_x3_kernel<true, true, true, 0,",
                    kernel="gemm_x3_kernel (fp32 as 3 bf16 planes x 6 MFMA products; peak = "
                           "dense bf16 2500 TF / 6)")
    return dict(mode="f32", peak=FP32_MFMA_PEAK_TFS, prefix="gemm_f32_kernel<true, true, true, 0,",
                kernel="gemm_f32_kernel (v_mfma_f32_32x32x2_f32)")


def gemm_dtype():
    """The bench line's `dtype`: the arithmetic the path computes in. Data and accumulation are
    fp32; the GEMMs run split arithmetics on the fp16 / bf16 matrix cores with fp32 accuracy."""
    from gatx import _lib
    mode = _lib.lib.gatx_get_gemm_mode()
    if mode == 2:
        gw = _lib.lib.gatx_gemm_layout_mode(0, 0)
        return ("fp32 (GEMMs: f16x3 split = 2 fp16 planes x 3 MFMA products, x3 fallback per "
                "out-of-range tile" + ("" if gw == 2 else "; weight gradient x3 = 3 bf16 planes x "
                                       "6 products") + ")")
    if mode == 1:
        return "fp32 (GEMMs: x3 split = 3 bf16 planes x 6 MFMA products)"
    return "fp32 (GEMMs: v_mfma_f32_32x32x2_f32)"


def run_timed(step, steps, world, dev, instr_step=None, instr_outside=False):
    """The timed region: barrier + synchronize on both sides, max over ranks. Returns (elapsed,
    per-kernel HIP-event records, instrumented step count). Only the last steps // 10 (>= 1)
    steps bracket their launches with HIP events on the launch stream: each timed event record
    costs the stream ~10 us (rocprof traces: 14-16 extra gaps per PPI step when every step was
    bracketed), so instrumenting every step would inflate the headline by 3-6%; this way the
    kernel timings are live, inside the timed region, at < 1% cost to it. With a captured
    hipGraph `step`, the instrumented steps run `instr_step` (the same step, eagerly): events
    bracket individual launches, which a graph replay does not expose.
    The region is bracketed by two gatx_region_mark dispatches (the first carries `steps` in its
    grid size) enqueued outside the clock, so a rocprofv3 counter pass can cut exactly these
    steps' dispatches out of its trace (tools/pmc_summary.py).
    instr_outside (launch-bound captured steps: PATTERN, Planetoid, training): all `steps` timed steps are
    graph replays and the instrumented eager steps run right after the clock stops — an eager
    step of ~80 small launches is host-bound (it took ~3x a replay), so inside the clock it would
    measure the Python launch path, not the step."""
    from gatx import _lib
    from gatx.functional import KernelTimer, set_kernel_timer
    n_instr = max(1, steps // 10)
    timer = KernelTimer()
    _lib.call("gatx_region_mark", steps, _lib.stream())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outside = instr_outside and instr_step is not None
    for i in range(steps):
        if i == steps - n_instr and not outside:
            set_kernel_timer(timer)
            if instr_step is not None:
                step = instr_step
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    set_kernel_timer(None)
    _lib.call("gatx_region_mark", 1, _lib.stream())
    if outside:
        set_kernel_timer(timer)
        for _ in range(n_instr):
            instr_step()
        torch.cuda.synchronize()
        set_kernel_timer(None)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, timer.summary(), n_instr


def layer_dims(cfg):
    heads = [1] + cfg["num_heads_per_layer"]
    widths = cfg["head_output_features_per_layer"]
    return [(heads[i] * widths[i], heads[i + 1], widths[i + 1], cfg["heads_concat_per_layer"][i])
            for i in range(cfg["num_layers"])]


def _r4(v):
    return (v + 3) // 4 * 4


def survey_bytes(N, E2, F_in, NH, F, concat):
    """SURVEY.md §8(d)'s per-layer formulas (fp32 = 4 B, int32 indices): B_gemm, FLOP_gemm and
    B_edge, which prices one Wh[src] row gather PER EDGE (no cache reuse credited). That is the
    traffic an L2-less machine would move, not HBM bytes: reported as `l2_gather_GBps` only."""
    b_gemm = 4 * (N * F_in + F_in * NH * F + N * NH * F + 2 * N * NH)
    f_gemm = 2 * N * F_in * NH * F + 4 * N * NH * NH * F
    b_edge = 4 * (2 * (E2 + N + 1) + 2 * (E2 * NH + N * NH) + E2 * NH * F + E2 * NH
                  + (N * NH * F if concat else N * F))
    return b_gemm, f_gemm, b_edge


def distinct_sources_per_chunk(graph, chunk):
    """Sum over the edge pass's node chunks (`chunk` consecutive destinations, the unit one XCD
    sweeps per head group: edge_fwd.hip's chunked items) of the distinct source ids their edges
    gather: the rows a chunk must bring from beyond the L2, read again by the next chunk only
    from the MALL or HBM. Device-side sort, once per graph, outside any timing."""
    E2 = graph.num_edges
    key = (graph.rowidx[:E2].to(torch.int64) // chunk) * graph.num_nodes \
        + graph.col[:E2].to(torch.int64)
    n = int(torch.unique(key).numel())
    del key
    return n


def layer_dataflow(N, E2, F_in, NH, F, concat, resid, alpha=True, gather_rows=None):
    """Per-kernel COMPULSORY bytes and flops of one gatx layer forward, following the dataflow the
    library actually runs (gatx.functional.layer_forward): the reassociated first layer gathers
    4*round4(F_in)-byte x rows, the others 4*NH*Fp-byte Wh rows. Gathered rows count once per
    node when the gathered matrix fits in the on-chip caches (<= the 256 MB MALL: every PPI /
    PATTERN / Planetoid batch), and once per EDGE when it does not (RMAT: 20 GB of Wh gathered
    in random order, so every gather is an HBM read; hub sources aside). Every other array is
    read or written once. alpha=False: the inference forward defers the alpha pass to the first
    read of normalised_attention_coeffs (gatx.functional.LazyAlpha), so a step that never reads
    it does not run it. gather_rows: the gathered-row count beyond the MALL when known
    (distinct_sources_per_chunk: a source's row is read once per node chunk that gathers it, not
    once per edge). Returns [(kernel, bytes, flops)]."""
    from gatx import tuning
    from gatx.functional import LayerShape, fold_scores_into_gemm, use_reassociation
    sh = LayerShape(NH, F, F_in, concat, False)
    H2, Fp, Dp = 2 * NH, sh.Fp, sh.Dp
    oc = sh.out_cols
    r = oc if resid else 0
    mx = ("attention_max", 4 * (2 * E2 + N * H2), 0)
    alpha = [("attention_alpha", 16 * E2 + 4 * (N * H2 + N * NH + E2 * NH), 0)] if alpha else []
    if use_reassociation(sh):
        Fin_p = _r4(F_in)
        gath = N * Fin_p if N * Fin_p * 4 <= MALL_BYTES else E2 * Fin_p
        return [
            ("gemm_scores", 4 * (N * F_in + H2 * F_in + N * H2), 2 * N * F_in * H2),
            mx,
            ("edge_forward", 4 * ((N + 1) + E2 + N * H2 + gath + N * NH * Fin_p + N * NH), 0),
            *alpha,
            ("gemm_out", 4 * (N * NH * Fin_p + NH * F * Fin_p + N * oc + N * r),
             2 * N * Fin_p * NH * F),
        ]
    gath = N * Dp if N * Dp * 4 <= MALL_BYTES else (gather_rows or E2) * Dp
    out = []
    if fold_scores_into_gemm(sh):
        out.append(("gemm", 4 * (N * F_in + (Dp + H2) * F_in + N * Dp + N * H2),
                    2 * N * F_in * (NH * F + H2)))
    elif tuning.get("fused_scores"):
        # S reduced from the accumulators in the GEMM epilogue (gatx_projection_gemm_scores): no
        # second read of Wh; flops counted as the 2NH extra columns of x W_aug^T
        out.append(("gemm", 4 * (N * F_in + (Dp + H2) * F_in + N * Dp + N * H2),
                    2 * N * F_in * (NH * F + H2)))
    else:
        out.append(("gemm", 4 * (N * F_in + Dp * F_in + N * Dp), 2 * N * F_in * NH * F))
        out.append(("node_scores", 4 * (N * Dp + N * H2), 2 * N * Dp * H2))
    out += [mx,
            ("edge_forward", 4 * ((N + 1) + E2 + N * H2 + gath + N * NH + N * oc + N * r), 0),
            *alpha]
    return out


def layer_backward_dataflow(N, E2, F_in, NH, F, concat, elu, need_x, fold_resid=False):
    """Per-kernel COMPULSORY bytes and flops of one gatx layer backward, following the dataflow
    gatx.functional.layer_backward runs (the closed-form autograd of models/gat_layer.py:64-135,
    SURVEY.md §8a a14). Phase names are the KernelTimer records the backward makes, so each
    record can be priced. Gathered rows (Wh, go) count once per node while the gathered matrix
    fits the 256 MB MALL, else once per edge; every other array once. The reassociated first layer
    whose input needs no gradient (the model input) takes _reassoc_backward's dataflow.
    fold_resid: the identity skip's gradient accumulated by the g_x GEMM (reads g_x once more).
    A folded Linear skip (PATTERN) is not modelled. Returns [(phase, bytes, flops)]."""
    from gatx.functional import LayerShape, use_reassociation
    sh = LayerShape(NH, F, F_in, concat, False)
    H2, Fp, Dp = 2 * NH, sh.Fp, sh.Dp
    oc = sh.out_cols
    go_w = Dp if concat else Fp
    g_out = 4 * N * oc * (2 if elu else 1)            # g_out (+ out for ELU's derivative)
    csr = 4 * ((N + 1) + 2 * E2)                      # rowptr / col / perm (or the transpose's)
    soft = 4 * (N * H2 + N * NH)                      # S and den
    if use_reassociation(sh) and not need_x:
        Fin_p = _r4(F_in)
        xg = N * Fin_p if N * Fin_p * 4 <= MALL_BYTES else E2 * Fin_p
        return [
            ("bwd_prepare_go", g_out + 4 * N * Dp, 0),
            ("bwd_gemm_gz", 4 * (N * Dp + NH * F * Fin_p + N * NH * Fin_p),
             2 * N * Fin_p * F * NH),
            ("bwd_edge_dst", csr + soft + 4 * (N * NH * Fin_p + xg + NH * E2 + 2 * N * NH), 0),
            ("bwd_src_scores", 4 * ((N + 1) + E2 + NH * E2 + N * NH), 0),
            ("bwd_max", 4 * N * NH, 0),
            ("bwd_gemm_gw_z", 4 * (N * Dp + N * NH * Fin_p + NH * F * F_in),
             2 * NH * F * F_in * N),
            ("bwd_gemm_gs", 4 * (N * H2 + N * F_in + H2 * F_in), 2 * H2 * F_in * N),
            ("bwd_weight_grads", 4 * ((sh.K_aug + NH * F) * F_in + 2 * NH * NH * 2 * F), 0),
        ]
    KC = sh.K_aug
    ldg = _r4(KC)
    wh = N * Dp if N * Dp * 4 <= MALL_BYTES else E2 * Dp
    gog = N * go_w if N * go_w * 4 <= MALL_BYTES else E2 * go_w
    out = [
        # (an identity skip's gradient is go itself: no extra array)
        ("bwd_prepare_go", g_out + 4 * N * go_w, 0),
        # g_alpha' per edge from go[n] . Wh[src], softmax backward: g_raw (NH x E2), g_s_dst
        ("bwd_edge_dst", csr + soft + 4 * (N * go_w + wh + NH * E2 + 2 * N * NH), 0),
        # message gradient sum alpha~ go[dst] and g_s_src, one G_aug row per source
        ("bwd_edge_src", csr + soft + 4 * (gog + NH * E2 + N * (Dp + NH)), 0),
        ("bwd_max", 4 * N * NH, 0),
    ]
    # G_aug's exact row / column maxima for the f16x3 gradient GEMMs' scales (one read)
    out.append(("bwd_gaug_stats", 4 * (N * ldg + N + KC), 0))
    if need_x:
        out.append(("bwd_gemm_gx", 4 * (N * ldg + 2 * KC * F_in + N * F_in
                                        + (N * F_in if fold_resid else 0)),
                    2 * N * F_in * KC))
    out += [("bwd_gemm_gw", 4 * (N * ldg + N * F_in + KC * F_in), 2 * KC * F_in * N),
            ("bwd_weight_grads", 4 * ((KC + NH * F) * F_in + 2 * NH * NH * 2 * F), 0)]
    return out


def graph_transpose_bytes(E2, N):
    """The backward's source-ordered CSR (graph_transpose): reads col / rowidx / perm, writes
    srowptr, scol, seid."""
    return 12 * E2 + 12 * E2 + 4 * (N + 1)


def train_step_dataflow(cfg, N, E, E2, n_params, build_graph=True):
    """Per-kernel compulsory bytes and flops of one PPI_GAT / PatternGAT-style training step as
    bench.py runs it: graph build (+ the backward's transpose), the forward with alpha (training
    forwards write it), the loss (fused BCE + its scaling backward), calc_attention_norm over the
    layers' alphas, the backward of every layer (the first layer's input needs no gradient), and
    the fused Adam update (param, grad, exp_avg, exp_avg_sq: 4 reads + 3 writes of 4 B per
    parameter). Returns [(phase, bytes, flops)]."""
    dims = layer_dims(cfg)
    L = len(dims)
    flows = []
    if build_graph:
        flows.append(("graph_build", graph_build_bytes(E, E2, N), 0))
        flows.append(("graph_transpose", graph_transpose_bytes(E2, N), 0))
    for i, (fin, nh, f, cc) in enumerate(dims):
        flows += layer_dataflow(N, E2, fin, nh, f, cc, cfg["add_skip_connection"][i])
    n_out = N * cfg["num_classes"]
    flows += [("bce", 12 * n_out, 0), ("bce_bwd", 8 * n_out, 0)]
    for (_, nh, _, _) in dims:   # alpha, the int64 destinations, rowptr
        flows.append(("attn_norm", 4 * E2 * nh + 8 * E2 + 4 * (N + 1), 0))
    for i, (fin, nh, f, cc) in enumerate(dims):
        skip = cfg["add_skip_connection"][i]
        ident = skip and fin == nh * f   # identity skip: folded into the g_x GEMM's accumulate
        flows += layer_backward_dataflow(N, E2, fin, nh, f, cc, elu=(i != L - 1),
                                         need_x=i > 0, fold_resid=ident)
    flows.append(("adam", 28 * n_params, 0))
    return flows


def edge_pricer(dims, flows):
    """edge_bytes(i, info) for roofline_objects: the compulsory bytes of the i-th edge_forward
    record of a step. Records come in layer order, one per layer (a head-mean layer's head-group
    launches share one record), so the layer is i mod the layer count; the record's head count
    must match that layer's."""
    def price(i, info):
        li = i % len(dims)
        if info[2] != dims[li][1]:
            raise KeyError(f"edge record {i} {info} does not match layer {li} {dims[li]}")
        return [bb for k, bb, _ in flows[li] if k == "edge_forward"][0]
    return price


def graph_build_bytes(E, E2, N):
    """Compulsory bytes of the per-step graph preprocessing: read edge_index (int64), write
    edge_index' (int64) and the int32 CSR (col, rowidx, perm, rowptr)."""
    return 16 * E + 16 * E2 + 12 * E2 + 4 * (N + 1)


def load_pmc(pm_path):
    """A committed tools/pmc_summary.py summary, or None (missing, or written before the
    region-marked window existed: such a summary cannot tell step kernels from setup kernels)."""
    if not os.path.exists(pm_path):
        return None
    pm = json.load(open(pm_path))
    return pm if "window" in pm else None


def pmc_step_bytes(pm, step_ms, pm_path=""):
    """Fabric bytes per step measured by rocprofv3 (FETCH_SIZE x 2 + WRITE_SIZE, the
    MI355X_MICROARCH.md gfx950 correction; Infinity-Cache hits are included, so this bounds HBM
    traffic from above): every dispatch between bench.py's two region marks, over the step count
    the first mark carries (tools/pmc_summary.py)."""
    if pm is None:
        return None
    from pmc_summary import step_bytes
    per_step = step_bytes(pm)
    gbs = per_step / (step_ms * 1e-3) / 1e9
    return {"bytes_per_step": per_step, "GBps": round(gbs, 1),
            "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4), "steps_in_window": pm["steps"],
            "source": f"{os.path.relpath(pm_path, ROOT)} ({pm.get('source', '')}); step time of "
                      "this run",
            "note": "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE (gfx950 correction) of the dispatches "
                    "between the timed region's marks; counts Infinity-Cache hits, so an upper "
                    "bound on HBM bytes"}


def available_cores():
    """Host cores this process may use: the affinity set, capped by a cgroup CPU quota if one is
    set (the GPU box grants each job a share of a larger machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = max(1, min(n, int(int(q) // int(per))))
    except Exception:
        pass
    return n


def _cpu_timer(fn, budget_s):
    times = []
    t_start = time.perf_counter()
    fn()   # warm-up
    while True:
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s or len(times) >= 3:
            break
    return min(times), len(times)


def cpu_baseline(model, cfg, ds, graphs, budget_s=20.0):
    """The reference's CPU dataflow restated in torch eager (oracle/torch_dataflow.py: index,
    cat, mm through `a`, max, exp, scatter_add_, exactly the ops of models/gat_layer.py:64-127)
    on `graphs` graphs of the same workload, every available host core."""
    from oracle import torch_dataflow as td
    from gatx import data as gd
    cores = available_cores()
    torch.set_num_threads(cores)
    b = gd.dataset_batch(ds, graphs, graph_seed=4242)
    dims = layer_dims(cfg)
    layers = [(l.W.weight.detach().cpu(), l.a.weight.detach().cpu()) for l in model.gat_layer_list]
    skips = [None if isinstance(s, torch.nn.Identity) else s.weight.detach().cpu()
             for s in model.skip_layer_list]
    x = torch.from_numpy(b.x)
    ei = torch.from_numpy(b.edge_index)
    res = {}

    def run():
        with torch.no_grad():
            res["o"] = td.model_forward(x, ei, layers, skips, cfg["num_heads_per_layer"],
                                        [d[2] for d in dims], cfg["heads_concat_per_layer"],
                                        cfg["add_skip_connection"])
    best, n = _cpu_timer(run, budget_s)
    e_tot = sum(a.shape[0] for a in res["o"][2])
    return {"value": e_tot / best, "unit": "layer-edges/s", "cores": cores, "kind": "port",
            "sample": f"torch-eager port of the reference dataflow (oracle/torch_dataflow.py),"
                      f" {ds} {len(dims)}-layer fwd on {graphs} graph(s) (N={b.num_nodes}, sum "
                      f"E'={e_tot}), {cores} threads, best of {n}: {best:.3f} s; the reference "
                      "itself, timed in the build container: bench/cpu_reference_baseline.json"}


def cpu_baseline_rmat(W, a, NH, F, budget_s=20.0):
    """The torch restatement on a scaled RMAT (1e5 nodes / 1.6e6 edges, SURVEY.md §8d 'RMAT on
    CPU'), one GATLayer forward (F_in 512 -> 8 x 64 concat)."""
    from oracle import torch_dataflow as td
    from gatx import data as gd
    cores = available_cores()
    torch.set_num_threads(cores)
    n, e = 100_000, 1_600_000
    ei = torch.from_numpy(gd.rmat_edges(n, e, seed=4242))
    x = torch.from_numpy(gd.normal(7, n * W.shape[1]).reshape(n, W.shape[1]))
    Wt, at = torch.from_numpy(W), torch.from_numpy(a)
    res = {}

    def run():
        with torch.no_grad():
            res["o"] = td.layer_forward(x, ei, Wt, at, NH, F, True)
    best, k = _cpu_timer(run, budget_s)
    E2 = res["o"][2].shape[0]
    return {"value": E2 / best, "unit": "layer-edges/s", "cores": cores, "kind": "port",
            "sample": f"torch-eager port of the reference dataflow, 1 GATLayer fwd on a "
                      f"SCALED RMAT (N={n}, E'={E2}; the full 1e7/1.6e8 graph is infeasible on "
                      f"CPU), {cores} threads, best of {k}: {best:.3f} s"}


def kernel_summary(summ, n_instr):
    kern = {}
    for phase, recs in summ.items():
        tot = sum(t for _, t in recs)
        kern[phase] = {"launches": len(recs), "avg_ms": tot / len(recs),
                       "total_ms_per_step": tot / n_instr}
    return kern


L2_GATHER_TBS = 17.8   # the guide's L2-resident row-gather rate (16.8-18.8 TB/s, MI355X_MICROARCH.md)


def _lds_record(info):
    """An edge_forward record of the LDS-staged pass (gatx.functional: info ends with "lds")."""
    return len(info) > 5 and info[5] == "lds"


def gathered_row_bytes(E2, info):
    """Bytes of source rows one edge_forward record gathers through L2 (one row per edge): the
    reassociated first layer's 4*round4(F_in)-byte x rows (info[4] == "x", info[3] = the padded
    width), else 4*NH*round4(F)-byte Wh rows."""
    if info[4] == "x":
        return 4 * E2 * info[3]
    return 4 * E2 * info[2] * _r4(info[3])


def roofline_objects(summ, edge_bytes, pm, n_instr, pm_path="", gather_E2=None):
    """The two roofline objects (projection GEMM: MFMA-bound; edge pass: HBM-bound), each priced
    per launch from the live HIP-event durations, the GEMM by its flops, the edge pass by its
    compulsory bytes: edge_bytes(i, info) prices the i-th edge_forward record of a step (records
    come in layer order, one per layer; layer_dataflow). `traffic` = the PMC-measured fabric bytes
    per step of the same kernel(s) (tools/pmc_summary.py window) divided by the records one step
    makes, i.e. per record like `achieved` (a head-mean layer's head groups are several launches
    inside one record)."""
    roofs = {}
    gem = summ.get("gemm", [])
    if gem:
        fl = sum(2.0 * n * fin * (nh * f + 2 * nh) for (n, _, fin, nh, f), _ in gem)
        ms_ = sum(t for _, t in gem)
        tfs = fl / (ms_ * 1e-3) / 1e12
        gr = gemm_roof()
        from gatx.functional import use_weight_planes
        label = gr["kernel"]
        if gr["mode"] == "f16x3" and not any(use_weight_planes(nh * f + 2 * nh, fin, n)
                                             for (n, _, fin, nh, f), _ in gem):
            # (small layers: the tiled / small-K / tiny kernels the library picks by shape)
            label = ("tiled / small-K GEMM kernels by shape, f16x3 arithmetic where tiled (peak "
                     "= dense fp16 2500 TF / 3)")
        roofs["gemm"] = {"bound": "mfma", "kernel": label + ", projection x.W_aug^T",
                         "achieved": round(tfs, 2), "peak": round(gr["peak"], 1),
                         "unit": "TFLOP/s", "frac": round(tfs / gr["peak"], 4), "traffic": None,
                         # the same fp32 flops against the native fp32 MFMA peak (context only:
                         # the split arithmetics run on the fp16 / bf16 matrix cores)
                         "frac_of_fp32_mfma_peak": round(tfs / FP32_MFMA_PEAK_TFS, 4),
                         "gemm_mode": gr["mode"], "flops_per_launch": fl / len(gem),
                         "avg_launch_ms": ms_ / len(gem), "_prefix": gr["prefix"], "_ms": ms_,
                         "_per_step": len(gem) / n_instr}
    edg = summ.get("edge_forward", [])
    if edg:
        by = [edge_bytes(i, info) for i, (info, _) in enumerate(edg)]
        ms_ = sum(t for _, t in edg)
        gbs = sum(by) / (ms_ * 1e-3) / 1e9
        roofs["edge_forward"] = {"bound": "hbm",
                                 "kernel": "edge passes, all layers (edge_forward_shared_kernel, "
                                           "edge_lds_kernel, edge_forward_kernel<*>)",
                                 "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                                 "bytes_per_launch": sum(by) / len(edg),
                                 "bytes_per_layer": by[:len(edg) // n_instr],
                                 "bytes_basis": "compulsory bytes: gathered rows once per node when "
                                                "the gathered matrix fits the 256 MB MALL, else "
                                                "once per edge; CSR, scores, den, output (+ "
                                                "residual) once",
                                 "avg_launch_ms": ms_ / len(edg),
                                 "_prefix": ("edge_forward", "edge_lds"), "_ms": ms_,
                                 "_per_step": len(edg) / n_instr}
        if gather_E2:
            # what bounds the pass in cache-resident batches: the per-edge row gathers served by
            # L2, against the guide's L2-gather rate
            # (records of the LDS-staged pass read their rows from LDS: not L2 gathers)
            gat = [(info, t) for info, t in edg if not _lds_record(info)]
            if gat:
                gb = sum(gathered_row_bytes(gather_E2, info) for info, _ in gat)
                g_tbs = gb / (sum(t for _, t in gat) * 1e-3) / 1e12
                roofs["edge_forward"]["l2_gather"] = {
                    "achieved": round(g_tbs, 2), "peak": L2_GATHER_TBS, "unit": "TB/s",
                    "frac": round(g_tbs / L2_GATHER_TBS, 4),
                    "basis": "the L2-gather passes only (not the LDS-staged one): one source row "
                             "per edge through L2 (4 NH round4(F) B, the reassociated layer "
                             "4 round4(F_in) B) / their mean launch time; peak = the guide's "
                             "L2-resident gather rate"}
    if pm is not None:
        from pmc_summary import prefix_bytes_per_step
        for r in roofs.values():
            b = prefix_bytes_per_step(pm, r["_prefix"])
            if b > 0:
                r["traffic"] = b / r["_per_step"]
                r["traffic_source"] = (f"{os.path.relpath(pm_path, ROOT) if pm_path else ''} "
                                       f"({pm.get('source', '')})")
    ordered = sorted(roofs.values(), key=lambda r: -r["_ms"])
    for r in ordered:
        for k in ("_prefix", "_ms", "_per_step"):
            r.pop(k)
    return ordered


# what each training-step record is priced as: the KernelTimer phase -> its bound and the rocprof
# kernel-name prefix(es) its launches carry (for `traffic`)
TRAIN_PHASES = {
    "gemm": ("mfma", None),
    # (pre-split f16x3 g_x / the in-loop kernel; the f16x3 weight gradient / its x3 form)
    "bwd_gemm_gx": ("mfma", ("gemm_f16p_kernel<16, 1", "gemm_f16p_kernel<32, 1",
                             "gemm_x3_kernel<true, true, true, 1,")),
    "bwd_gemm_gw": ("mfma", ("gemm_f16rc_kernel<", "gemm_x3_kernel<false, false, true, 2, 1>")),
    "edge_forward": ("hbm", ("edge_forward", "edge_lds")),
    "bwd_edge_dst": ("hbm", "edge_bwd_dst"),
    "bwd_edge_src": ("hbm", "edge_bwd_src"),
    "bwd_prepare_go": ("hbm", "prepare_go"),
}


def gemm_phase_roof(phase):
    """(arithmetic, peak TF/s) of the GEMM a training record runs: the forward projection and g_x
    (both operands k-contiguous) in the active mode; the weight gradient G_aug^T x (row-contiguous
    operands) in the arithmetic the library reports for that layout."""
    from gatx import _lib
    gr = gemm_roof()
    if phase == "bwd_gemm_gw":
        mode = _lib.lib.gatx_gemm_layout_mode(0, 0)
        return {2: "f16x3", 1: "x3", 0: "f32"}[mode], {
            2: BF16_MFMA_PEAK_TFS / F16X3_PRODUCTS, 1: BF16_MFMA_PEAK_TFS / X3_PRODUCTS,
            0: FP32_MFMA_PEAK_TFS}[mode]
    return gr["mode"], gr["peak"]


def record_pricer(dims, flows, cfg):
    """price(phase, i, info) -> (bytes, flops) of the i-th record of `phase` in a training step:
    forward records from layer_dataflow (the projection GEMM by its flops; edge records by layer
    index), backward records from layer_backward_dataflow at the record's own shape (the info
    tuple functional.layer_backward records: N, E2, F_in, NH, F, concat, C, elu, reassoc[, fold])."""
    edge = edge_pricer(dims, flows)

    def price(phase, i, info):
        if phase == "gemm":
            n, _, fin, nh, f = info
            return 0, 2.0 * n * fin * (nh * f + 2 * nh)
        if phase == "edge_forward":
            return edge(i, info), 0
        N, E2, fin, nh, f, cc, _, elu, reassoc = info[:9]
        fold = bool(info[9]) if len(info) > 9 else False
        for k, b, fl in layer_backward_dataflow(N, E2, fin, nh, f, cc, elu, need_x=not reassoc,
                                                fold_resid=fold):
            if k == phase:
                return b, fl
        raise KeyError(f"{phase} record {info} not in the backward dataflow")
    return price


def train_gathered_row_bytes(phase, E2, info):
    """Source rows one training edge record gathers through L2, one row per edge and head (None
    for records not priced this way): the forward as gathered_row_bytes; the backward's
    destination pass reads Wh[src] per (edge, head) (4 round4(F) B), its source pass go[dst] per
    edge for every head of a concat layer and once for a head-mean one (go is then shared by the
    heads). The reassociated first layer's backward is not priced (its rows are x's)."""
    if phase == "edge_forward":
        return None if _lds_record(info) else gathered_row_bytes(E2, info)
    _, _, _, nh, f, cc = info[:6]
    if len(info) > 8 and info[8]:
        return None
    if phase == "bwd_edge_dst":
        return 4 * E2 * nh * _r4(f)
    if phase == "bwd_edge_src":
        return 4 * E2 * (nh if cc else 1) * _r4(f)
    return None


def train_roofline_objects(summ, price, pm, n_instr, pm_path="", gather_E2=None):
    """Roofline objects of a training step: every TRAIN_PHASES phase with records, priced per
    record (price(phase, i, info)) and timed by its HIP events; the two with the most time per
    step come first. GEMM phases are MFMA-bound (flops / the peak of the arithmetic they run),
    the others HBM-bound (compulsory bytes / 8 TB/s). `traffic` = PMC fabric bytes per record of
    the phase's kernels (tools/pmc_summary.py window of a train run), when a summary is given."""
    objs = []
    for phase, (bound, prefix) in TRAIN_PHASES.items():
        recs = summ.get(phase, [])
        if not recs:
            continue
        ms_ = sum(t for _, t in recs)
        priced = [price(phase, i, info) for i, (info, _) in enumerate(recs)]
        per_step = len(recs) / n_instr
        if bound == "mfma":
            fl = sum(f for _, f in priced)
            tfs = fl / (ms_ * 1e-3) / 1e12
            mode, peak = gemm_phase_roof(phase)
            o = {"bound": "mfma", "kernel": f"{phase} ({mode} arithmetic)", "achieved": round(tfs, 2),
                 "peak": round(peak, 1), "unit": "TFLOP/s", "frac": round(tfs / peak, 4),
                 "traffic": None, "gemm_mode": mode, "flops_per_launch": fl / len(recs)}
        else:
            by = sum(b for b, _ in priced)
            gbs = by / (ms_ * 1e-3) / 1e9
            o = {"bound": "hbm", "kernel": phase, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                 "bytes_per_launch": by / len(recs)}
        o.update({"avg_launch_ms": ms_ / len(recs), "records_per_step": per_step,
                  "ms_per_step": ms_ / n_instr})
        if gather_E2 and phase in ("edge_forward", "bwd_edge_dst", "bwd_edge_src"):
            # the bound of these passes in cache-resident batches: the per-edge row gathers from
            # L2, against the guide's L2-gather rate (records of unpriced layers left out)
            pr = [(train_gathered_row_bytes(phase, gather_E2, info), t) for info, t in recs]
            pr = [(b, t) for b, t in pr if b is not None]
            if pr:
                g_tbs = sum(b for b, _ in pr) / (sum(t for _, t in pr) * 1e-3) / 1e12
                o["l2_gather"] = {"achieved": round(g_tbs, 2), "peak": L2_GATHER_TBS,
                                  "unit": "TB/s", "frac": round(g_tbs / L2_GATHER_TBS, 4),
                                  "basis": "one gathered row per edge (and head): Wh[src] in the "
                                           "forward and the destination pass, go[dst] in the "
                                           "source pass; the reassociated first layer and the "
                                           "LDS-staged pass (rows from LDS) excluded"}
        if pm is not None and prefix:
            from pmc_summary import prefix_bytes_per_step
            b = prefix_bytes_per_step(pm, prefix)
            if b > 0:
                o["traffic"] = b / per_step
                o["traffic_source"] = (f"{os.path.relpath(pm_path, ROOT) if pm_path else ''} "
                                       f"({pm.get('source', '')}), kernels "
                                       + " | ".join(f"{x}*" for x in (prefix if isinstance(prefix, tuple) else (prefix,))))
        objs.append(o)
    return sorted(objs, key=lambda o: -o["ms_per_step"])


def run_rmat(args, world, rank, dev):
    """BASELINE config 5: one GATLayer (F_in 512 -> 8 heads x 64, concat, self-loops) forward on
    a synthetic R-MAT graph (1e7 nodes, exactly 1.6e8 edges), eval mode, CSR built per step. One
    graph, no sharding: with --gpus N each rank runs an independent replica (value sums them)."""
    from gatx import GATLayer, clear_graph_cache
    from gatx import data as gd
    NH, F, FIN = 8, 64, 512
    N, E = args.rmat_nodes, args.rmat_edges
    torch.manual_seed(0)
    train = args.mode == "train"
    layer = GATLayer(FIN, F, NH, True, add_self_loops=True).to(dev).train(train)
    ei = gd.rmat_edges_device(N, E, seed=42 + rank, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1 + rank)
    x = torch.randn(N, FIN, device=dev, generator=g)
    gout = None
    if train:
        # a middle layer's backward: gradients for x, W and a from a fixed upstream gradient
        # (the hub-split backward passes, SURVEY.md §7 degree skew, on the power-law graph)
        x.requires_grad_(True)
        gout = torch.randn(N, NH * F, device=dev, generator=g)

    def step():
        clear_graph_cache()
        if train:
            layer.zero_grad(set_to_none=True)
            x.grad = None
            out = layer(x, ei)
            out.backward(gout)
            return out
        with torch.no_grad():
            return layer(x, ei)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    from gatx.graph import graph_cache
    E2 = graph_cache.get(ei, N, True).num_edges
    elapsed, summ, n_instr = run_timed(step, args.steps, world, dev)
    step_s = elapsed / args.steps
    # gathered Wh rows (20 GB of them, far beyond the MALL): a source's row comes from HBM once
    # per destination chunk that gathers it (R-MAT hubs are gathered by almost every chunk, but
    # re-read within one only from L2), not once per edge
    from gatx import tuning
    chunk = tuning.get("edge_chunk")
    g_rows = distinct_sources_per_chunk(graph_cache.get(ei, N, True), chunk)
    flow = layer_dataflow(N, E2, FIN, NH, F, True, False, gather_rows=g_rows)
    uniq = sum(b for _, b, _ in flow) + graph_build_bytes(E, E2, N)
    peak = gemm_roof()["peak"] * 1e12
    t_roof = sum(max(b / (HBM_PEAK_GBS * 1e9), f / peak) for _, b, f in flow) \
        + graph_build_bytes(E, E2, N) / (HBM_PEAK_GBS * 1e9)
    b_gemm, _, b_edge = survey_bytes(N, E2, FIN, NH, F, True)
    edge_b = [b for k, b, _ in flow if k == "edge_forward"][0]
    pmc_path = os.path.join(ROOT, "profiles", "pmc_rmat.json")
    pm = load_pmc(pmc_path) if not train else None   # the committed counters are forward-only
    roofs = roofline_objects(summ, lambda i, info: edge_b, pm, n_instr, pmc_path)
    result = {
        "metric": "GAT-layer edges/sec + achieved HBM GB/s, RMAT 1-layer fwd"
                  + (" (+bwd)" if train else ""),
        "value": round(E2 * world / step_s, 1), "unit": "layer-edges/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": gemm_dtype(),
        "data": "synthetic R-MAT (a,b,c,d)=(0.57,0.19,0.19,0.05), rejected ids redrawn, ids "
                "permuted, x ~ N(0,1), xavier weights",
        "config": {"workload": f"RMAT {N} nodes / {E} edges, GATLayer 512 -> 8x64 concat, "
                               f"self-loops, {'fwd+bwd' if train else 'eval'}, CSR built per step",
                   "gathered_rows_per_layer": g_rows,
                   "gather_model": f"a source row once per {chunk}-destination chunk that "
                                   "gathers it (distinct_sources_per_chunk), not once per edge",
                   "hub_split_backward": train and tuning.get("bwd_hubs") != 0,
                   "nodes": N, "edges_in": int(ei.size(1)), "edges_per_layer": E2,
                   "parallelism": "replicas" if world > 1 else "single GPU"},
        "unique_GBps": round(uniq / step_s / 1e9, 1),
        "roofline_time_frac": None if train else round(t_roof / step_s, 4),
        "l2_gather_GBps": round((b_gemm + b_edge) / step_s / 1e9, 1),
        "hbm_measured": None if train else pmc_step_bytes(pm, step_s * 1e3, pmc_path),
        "roofline": roofs[0] if roofs else None,
        "roofline_other": roofs[1] if len(roofs) > 1 else None,
        "kernels": kernel_summary(summ, n_instr),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not train:
        result["cpu_baseline"] = cpu_baseline_rmat(layer.W.weight.detach().cpu().numpy(),
                                                   layer.a.weight.detach().cpu().numpy(), NH, F)
    result["config"]["tuning"] = tuning_changes()
    if rank == 0:
        print(json.dumps(result), flush=True)


def launch_command(nproc: int, argv, port: int):
    """The torch.distributed.run command that starts `nproc` ranks of this script with the same
    arguments (one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__), *argv]


def launch_ranks(nproc: int, argv) -> int:
    """`bench.py --gpus N` started as ONE process (the driver's command form): start N fresh rank
    processes under torch.distributed.run as children, before this process touches the GPU (no
    exec: it would be forbidden after GPU init, and is not needed), relay their stdout (rank 0's
    JSON line) and return their exit status (non-zero if any rank failed)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    proc = subprocess.run(launch_command(nproc, argv, port), stdout=subprocess.PIPE, text=True)
    sys.stdout.write(proc.stdout)
    sys.stdout.flush()
    if proc.returncode != 0:
        print(f"bench.py: {nproc}-rank run failed with exit status {proc.returncode}",
              file=sys.stderr)
    return proc.returncode


def tuning_changes() -> dict:
    """The gatx.tuning switches this run set away from their defaults (--tune)."""
    from gatx import tuning
    cur = tuning.current()
    return {k: v for k, v in cur.items() if v != tuning.DEFAULTS[k]}


def dry_run(args, world: int, rank: int, local: int) -> int:
    """`--dry-run`: the multi-rank launch and timing protocol without a GPU. Each rank checks
    WORLD_SIZE == --gpus, joins a gloo group on 127.0.0.1, runs warmup + steps empty steps
    bracketed by barriers, and the elapsed time is max-reduced over ranks exactly as run_timed
    does; rank 0 prints one JSON line naming every rank that reported (its RANK / LOCAL_RANK)."""
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        dist.init_process_group("gloo")
    for _ in range(args.warmup):
        pass
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ranks = [[rank, local]]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ranks = [None] * world
        dist.all_gather_object(ranks, [rank, local])
    if rank == 0:
        print(json.dumps({"metric": "dry run (launch path only, no GPU)", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed / max(args.steps, 1) * 1e3, "ranks": ranks,
                          "dry_run": True}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def replay_check(replay, eager, out, alphas, eager_alphas, x, x_alt):
    """Proof that a replay of the captured step does its work (verdict r5: a stale node-block
    count once made the LDS pass skip its work on every timed replay, invisible because the
    buffers still held the previous replay's results). The static input x is replaced by x_alt,
    the captured step's static output and every layer's static alpha are poisoned with NaN by
    launches outside the graph (what triggered that bug), the graph is replayed once and its
    output / alphas compared BITWISE with an eager step on x_alt; x is restored after. A pass
    that skips its work leaves NaN or values of the old input in some layer, and every later layer
    inherits them. Returns (ok, detail)."""
    keep = x.clone()
    try:
        x.copy_(x_alt)
        out.fill_(float("nan"))
        for a in alphas:
            a.fill_(float("nan"))
        replay()
        got_out = out.clone()
        got_al = [a.clone() for a in alphas]
        ref_out = eager().clone()
        ref_al = eager_alphas()
        if x.is_cuda:
            torch.cuda.synchronize()
        bad = []
        if not torch.equal(got_out, ref_out):
            bad.append("output")
        for i, (g, r) in enumerate(zip(got_al, ref_al)):
            n = r.shape[0]
            if g.shape[0] < n or not torch.equal(g[:n], r):
                bad.append(f"alpha[{i}]")
        return not bad, ("bitwise equal to an eager step" if not bad
                         else "differs from an eager step: " + ", ".join(bad))
    finally:
        x.copy_(keep)


def train_leg_command(args) -> list:
    """The default forward run's second leg (BASELINE config 3, PPI 3-layer fwd+bwd train step,
    models/ppi_gat.py:15-33): this bench in --mode train as a child process (its own model,
    optimizer and captured step), with the same steps / warmup / graphs / tuning switches."""
    cmd = [sys.executable, os.path.abspath(__file__), "--mode", "train", "--no-cpu-baseline",
           "--no-train-leg", "--steps", str(args.steps), "--warmup", str(args.warmup)]
    if args.graphs is not None:
        cmd += ["--graphs", str(args.graphs)]
    for t in args.tune:
        cmd += ["--tune", t]
    return cmd


def train_leg_keys(line: dict) -> dict:
    """The train leg's figures as extra keys of the forward line (never `value`)."""
    return {"train_ms_per_step": line["ms_per_step"],
            "train_value": line["value"],
            "train_unit": line["unit"],
            "train_roofline_time_frac": line.get("roofline_time_frac"),
            "train_roofline": line.get("roofline"),
            "train_workload": line["config"]["workload"],
            "train_launch": line["config"].get("launch")}


def run_train_leg(args) -> dict:
    import subprocess
    proc = subprocess.run(train_leg_command(args), stdout=subprocess.PIPE, text=True,
                          timeout=900)
    if proc.returncode != 0:
        raise SystemExit(f"bench.py: the train leg failed (rc {proc.returncode})")
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    return train_leg_keys(json.loads(lines[-1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graphs", type=int, default=None,
                    help="graphs per rank (PPI default 20, PATTERN default 32)")
    ap.add_argument("--mode", choices=["fwd", "train"], default="fwd")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--attention-penalty", type=float, default=0.0,
                    help="PPI_GAT attention_penalty (train mode)")
    ap.add_argument("--attention-reward", type=float, default=0.0,
                    help="PlanetoidGAT attention_reward (train mode; the norm term is always added)")
    ap.add_argument("--workload", choices=["ppi", "pattern", "rmat", "cora", "citeseer",
                                           "pubmed"], default="ppi",
                    help="ppi: the BASELINE metric; pattern: config 4 (batch-sharded PATTERN "
                         "training); rmat: config 5; cora/citeseer/pubmed: the transductive "
                         "PlanetoidGAT step (one graph; with --gpus N, N replicas)")
    ap.add_argument("--rmat-nodes", type=int, default=10_000_000)
    ap.add_argument("--rmat-edges", type=int, default=160_000_000)
    ap.add_argument("--cached-graph", action="store_true",
                    help="reuse the CSR across steps (excludes graph preprocessing)")
    ap.add_argument("--wiring", choices=["gatx", "reference"], default="gatx",
                    help="gatx: skip / ELU / dropout fused into the layers; reference: the "
                         "reference GATModel.forward op for op around gatx GATLayers (the "
                         "INTEGRATION.md drop-in)")
    ap.add_argument("--tune", action="append", default=[], metavar="SWITCH=VALUE",
                    help="set a gatx.tuning switch for this run (A/B measurements; repeatable); "
                         "the line's config.tuning lists every switch that differs from default")
    ap.add_argument("--verify", action="store_true",
                    help="after timing, compare one more timed-path step's output with an eager "
                         "step's (stderr; diagnostic)")
    ap.add_argument("--no-train-leg", action="store_true",
                    help="skip the forward run's train-step leg (train_* keys; a child "
                         "bench.py --mode train, N=1 only)")
    ap.add_argument("--dry-run", action="store_true",
                    help="exercise the launch path only: --gpus N starts N ranks, each joins a "
                         "gloo group and runs the barrier / max-over-ranks timing around an empty "
                         "step, no GPU touched (CPU rehearsal of the driver's N-GPU command)")
    ap.add_argument("--hipgraph", choices=["auto", "on", "off"], default="auto",
                    help="replay each step as one captured hipGraph (gatx.capture). auto: forward "
                         "steps, and every training step on one GPU")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU over RCCL. Test-only overrides (exercise the multi-rank logic on a
    # one-GPU box): GATX_BENCH_BACKEND=gloo, GATX_BENCH_ONE_DEVICE=1 (every rank on cuda:0).
    if args.dry_run:
        sys.exit(dry_run(args, world, rank, local))
    from gatx import tuning
    tuning.set(**tuning.parse(args.tune))
    one_device = os.environ.get("GATX_BENCH_ONE_DEVICE") == "1"
    dev_idx = 0 if one_device else local
    backend = os.environ.get("GATX_BENCH_BACKEND", "nccl")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if not one_device and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: {world} ranks need {world} visible GPUs, "
                         f"{torch.cuda.device_count()} visible")
    if world > 1:
        torch.cuda.set_device(dev_idx)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev_idx}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{dev_idx}")
    if args.workload == "rmat":
        run_rmat(args, world, rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    from gatx import GATModel, clear_graph_cache
    from gatx import data as gd
    from gatx.config import data_config
    from gatx.distributed import GradientAllReducer, count_weights

    ds = {"pattern": "PATTERN", "ppi": "PPI", "cora": "Cora", "citeseer": "Citeseer",
          "pubmed": "Pubmed"}[args.workload]
    planetoid = ds in ("Cora", "Citeseer", "Pubmed")
    if planetoid:
        # transductive: one graph, trained every step (models/planetoid_gat.py); the edge list
        # never changes, so its CSR is built once and cached, as it is for any user of the layer
        args.graphs = 1
        args.cached_graph = True
    if args.graphs is None:
        args.graphs = 32 if ds == "PATTERN" else 20
    cfg = dict(data_config[ds])
    torch.manual_seed(0)
    model = GATModel(**cfg).to(dev)
    model.fuse_wiring = args.wiring == "gatx"
    model.train(args.mode == "train")
    b = gd.dataset_batch(ds, args.graphs, graph_seed=42 + 1000 * rank, feature_seed=1 + rank)
    x = torch.from_numpy(b.x).to(dev)
    ei = torch.from_numpy(b.edge_index).to(dev)
    y = (torch.rand(b.num_nodes, cfg["num_classes"], device=dev) > 0.5).float()
    train_mask = None
    if planetoid:
        # PlanetoidGAT (models/planetoid_gat.py:8-31): cross-entropy over the train split (PyG's
        # public split: 20 labelled nodes per class) plus attention_reward x the attention norm
        y = torch.randint(0, cfg["num_classes"], (b.num_nodes,), device=dev,
                          generator=torch.Generator(device=dev).manual_seed(3))
        train_mask = torch.zeros(b.num_nodes, dtype=torch.bool, device=dev)
        train_mask[:20 * cfg["num_classes"]] = True
        # out[mask] == out.index_select(0, mask.nonzero()): the same rows in the same order,
        # without the host sync a boolean index costs (the step stays capturable)
        train_idx = train_mask.nonzero().squeeze(1)
        y_train = y.index_select(0, train_idx)
        from gatx.graph import graph_cache as _gc
        _ = _gc.get(ei, b.num_nodes, True).num_edges   # built and validated before any capture
    use_graph = args.hipgraph == "on" or (
        args.hipgraph == "auto" and (args.mode == "fwd" or world == 1))
    if use_graph and args.mode == "train" and not args.cached_graph and ds != "PATTERN":
        # PPI_GAT's step returns the attention (forward_and_return_attention) while its CSR is
        # rebuilt every step: promise |edge_index'| (known from one eager build of this batch)
        # so the captured step needs no device read (gatx.graph.expect_num_edges)
        from gatx.graph import expect_num_edges, graph_cache as _gc
        expect_num_edges(ei, b.num_nodes, True, _gc.get(ei, b.num_nodes, True).num_edges)
    # a captured training step needs the optimizer's step counter on the device
    # torch's fused Adam (one launch for all parameters; same update rule as the reference's
    # Adam, models/*_gat.py configure_optimizers); a captured step needs capturable state
    opt = torch.optim.Adam(model.parameters(), lr=cfg["learning_rate"], fused=True,
                           weight_decay=cfg["l2_reg"],
                           capturable=use_graph and args.mode == "train")
    # PPI_GAT's nn.BCEWithLogitsLoss (models/ppi_gat.py:11,19) on gatx's fused loss kernels
    # (gatx.losses: one launch forward, one backward, instead of ~19 torch launches)
    from gatx.losses import BCEWithLogitsLoss
    loss_fn = BCEWithLogitsLoss()
    if planetoid:
        loss_fn = torch.nn.CrossEntropyLoss(reduction="mean")
    if ds == "PATTERN":   # PatternGAT (models/pattern_gat.py:11-15): class-balanced BCE
        loss_fn = BCEWithLogitsLoss(pos_weight=1 / 0.1765)
        y = y[:, 0].contiguous()
    reducer = None
    w_main = w_norm = 1.0
    if args.mode == "train" and world > 1:
        # DDP-style: buckets all-reduced (SUM) over RCCL as backward produces them; each rank's
        # mean loss terms weighted by its share of the union batch's counts:
        # nodes (labelled rows for Planetoid) for the BCE / CE, edges E' for the attention norm
        # (a per-edge mean). Counted once here, outside the timed / captured step.
        from gatx.graph import graph_cache as _gc
        e_local = _gc.get(ei, b.num_nodes, True).num_edges
        n_local = int(train_mask.sum()) if planetoid else b.num_nodes
        reducer = GradientAllReducer(model.parameters(), average=False)
        w_main, w_norm = count_weights([n_local, e_local],
                                       device=dev if backend == "nccl" else "cpu")

    from gatx.functional import _span
    n_params = sum(p.numel() for p in model.parameters())

    def _w(t, w):   # no extra launch for the single-rank weight 1
        return t if w == 1.0 else t * w

    # the loss's seed gradient, made once: backward() on a scalar would fill a fresh ones tensor
    # every step (one launch)
    one = torch.ones((), device=dev)

    def step():
        if not args.cached_graph:
            clear_graph_cache()
        if args.mode == "fwd":
            with torch.no_grad():
                return model(x, ei)
        opt.zero_grad(set_to_none=True)
        if ds == "PATTERN":   # PatternGAT.training_step (models/pattern_gat.py:18-25)
            out = model(x, ei).squeeze(-1)
            loss = _w(loss_fn(out, y), w_main)
        elif planetoid:       # PlanetoidGAT.training_step (models/planetoid_gat.py:15-31)
            out, ei2, atts = model.forward_and_return_attention(x, ei)
            attention_norm = model.calc_attention_norm(ei2, atts)
            loss = (_w(loss_fn(out.index_select(0, train_idx), y_train), w_main)
                    + args.attention_reward * w_norm * attention_norm)
        else:
            # PPI_GAT.training_step (models/ppi_gat.py:15-33): BCE + the attention norm, computed
            # every step (logged; added to the loss only with a non-zero attention_penalty)
            out, ei2, atts = model.forward_and_return_attention(x, ei)
            loss = _w(loss_fn(out, y), w_main)
            attention_norm = model.calc_attention_norm(ei2, atts)
            if args.attention_penalty != 0.0:
                loss = loss + args.attention_penalty * w_norm * attention_norm
        loss.backward(one)
        if reducer is not None:
            reducer.finish()
        with _span("adam", (n_params,)):
            opt.step()
        return out

    eager_step = step
    from gatx.capture import CapturedStep
    static_att = None
    if use_graph:
        step = CapturedStep(eager_step)
        # the captured forward's static alphas (each layer's (graph, alpha) as the capture left
        # it; later eager steps rebind the layers' attributes), for the replay check
        static_att = [l.__dict__.get("_attention") for l in model.gat_layer_list]
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    from gatx.graph import graph_cache
    N = b.num_nodes
    dims = layer_dims(cfg)

    from gatx import _lib
    fb = torch.zeros(1, dtype=torch.int64, device=dev)
    _lib.call("gatx_gemm_fallback_read", _lib.ptr(fb), 1, _lib.stream())   # reset the counter
    # launch-bound eager steps run their HIP-event instrumentation after the clock: small batches,
    # and every training step (autograd + ~110 launches: the eager PPI-20 step is host-bound,
    # ~1 ms of launch gaps in rocprof traces, so inside the clock it timed the Python path)
    instr_outside = use_graph and (args.mode == "train" or ds != "PPI" or args.graphs < 20)
    elapsed, summ, n_instr = run_timed(step, args.steps, world, dev,
                                       step.eager if use_graph else None, instr_outside)
    _lib.call("gatx_gemm_fallback_read", _lib.ptr(fb), 1, _lib.stream())
    fallback_tiles = int(fb.item())
    replay_verified = None
    replay_detail = None
    if use_graph and args.mode == "fwd" and static_att and all(
            a is not None and isinstance(a[1], torch.Tensor) for a in static_att):
        gen = torch.Generator(device=dev).manual_seed(2024 + rank)
        x_alt = torch.randn(x.shape, generator=gen, device=dev, dtype=x.dtype)

        def _eager_alphas():
            return [l.normalised_attention_coeffs.clone() for l in model.gat_layer_list]
        replay_verified, replay_detail = replay_check(
            step.graph.replay, step.eager, step.out, [a for _, a in static_att], _eager_alphas,
            x, x_alt)
    if args.verify and args.mode == "fwd":
        from gatx.graph import graph_cache as _gcv
        o1 = step().clone()
        torch.cuda.synchronize()
        _g = _gcv.get(ei, b.num_nodes, True)   # the captured step's graph (no eager step since)
        _h = _g._hub_plans.get(("blocks", 2304))
        print(f"bench.py --verify: node blocks after a timed-path step: "
              f"{int(_h[1].item()) if _h is not None else None}", file=sys.stderr)
        o2 = (step.eager if use_graph else eager_step)().clone()
        print(f"bench.py --verify: max|timed-path step - eager step| = "
              f"{float((o1 - o2).abs().max()):.3e}", file=sys.stderr)
    step_s = elapsed / args.steps
    ms = step_s * 1e3

    # the headline forward writes alpha in every layer, as the reference does
    # (models/gat_layer.py:106-110). For reference only, the same forward is also timed with
    # gatx's opt-in GATLayer.lazy_alpha (alpha computed on its first read, never read here):
    # reported as ms_per_step_alpha_deferred, never as value.
    alpha_deferred_ms = None
    if args.mode == "fwd" and world == 1:
        from gatx import GATLayer as _GL
        _GL.lazy_alpha = True
        st = CapturedStep(eager_step) if use_graph else eager_step
        for _ in range(args.warmup):
            st()
        el, _, _ = run_timed(st, args.steps, world, dev, st.eager if use_graph else None,
                             instr_outside)
        alpha_deferred_ms = el / args.steps * 1e3
        _GL.lazy_alpha = False
        del st

    clear_graph_cache()
    E2 = graph_cache.get(ei, N, True).num_edges
    layer_edges = len(dims) * E2
    value = layer_edges * world / step_s

    # honest accounting: unique bytes of the dataflow actually run, priced against HBM
    peak = gemm_roof()["peak"] * 1e12
    flows = [layer_dataflow(N, E2, fin, nh, f, cc, cfg["add_skip_connection"][i])
             for i, (fin, nh, f, cc) in enumerate(dims)]
    gb = graph_build_bytes(b.num_edges, E2, N) if not args.cached_graph else 0
    if args.mode == "train":
        # the whole training step: forward (alpha eager), loss, attention norm, backward, Adam
        tflow = train_step_dataflow(cfg, N, b.num_edges, E2, n_params,
                                    build_graph=not args.cached_graph)
        uniq = sum(bb for _, bb, _ in tflow)
        t_roof = sum(max(bb / (HBM_PEAK_GBS * 1e9), ff / peak) for _, bb, ff in tflow)
    else:
        uniq = sum(bb for fl in flows for _, bb, _ in fl) + gb
        t_roof = sum(max(bb / (HBM_PEAK_GBS * 1e9), ff / peak) for fl in flows
                     for _, bb, ff in fl) + gb / (HBM_PEAK_GBS * 1e9)
    surv = [survey_bytes(N, E2, fin, nh, f, cc) for (fin, nh, f, cc) in dims]
    l2_gather = sum(bg + be for bg, _, be in surv)

    edge_unique = edge_pricer(dims, flows)
    pm_name = "_none_"
    if ds == "PPI" and args.graphs == 20:
        pm_name = "pmc_latest.json" if args.mode == "fwd" else "pmc_train.json"
    pmc_path = os.path.join(ROOT, "profiles", pm_name)
    pm = load_pmc(pmc_path)
    if args.mode == "train" and ds == "PPI":
        ordered = train_roofline_objects(summ, record_pricer(dims, flows, cfg), pm, n_instr,
                                         pmc_path, gather_E2=E2)
    else:
        ordered = roofline_objects(summ, edge_unique, pm, n_instr, pmc_path, gather_E2=E2)

    result = {
        "metric": f"GAT-layer edges/sec + achieved HBM GB/s, {ds} {len(dims)}-layer fwd"
                  + ("" if args.mode == "fwd" else " (+bwd, train step)"),
        "value": round(value, 1), "unit": "layer-edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": gemm_dtype(),
        "data": f"synthetic {ds}-shaped graphs (uniform random edges, N(0,1) features), xavier "
                "weights",
        "config": {"workload": f"{ds} {len(dims)}-layer GAT {args.mode} ("
                               + "/".join(str(d[1]) for d in dims) + " heads, "
                               + "/".join(str(d[2]) for d in dims) + f"), "
                               f"{args.graphs} graphs per GPU"
                               + (", CSR cached" if args.cached_graph else ", CSR built per step"),
                   "graphs_per_gpu": args.graphs, "nodes_per_gpu": N, "edges_per_layer": E2,
                   "parallelism": ("replicas" if planetoid and world > 1
                                   else f"graph-batch dp{world}"),
                   "launch": ("eager" if not use_graph else
                              "hipGraph replay; kernel times from steps//10 HIP-event-instrumented "
                              "eager steps run after the clock (launch-bound)" if instr_outside
                              else "hipGraph replay (last steps//10 eager, HIP-event "
                                   "instrumented)"),
                   "wiring": ("gatx (skip / ELU / dropout fused into the layers)"
                              if args.wiring == "gatx" else
                              "reference GATModel.forward around gatx GATLayers (drop-in)"),
                   "alpha": "eager: every layer writes alpha in the forward, as the reference"},
        "ms_per_step_alpha_deferred": (round(alpha_deferred_ms, 4)
                                       if alpha_deferred_ms is not None else None),
        "gemm_f16x3_fallback_tiles_per_step": fallback_tiles / args.steps,
        "unique_GBps": round(uniq / step_s / 1e9, 1),
        "roofline_time_frac": (round(t_roof / step_s, 4) if ds == "PPI" or args.mode == "fwd"
                               else None),
        "roofline_time_basis": ("sum over the forward's kernels of max(unique bytes / 8 TB/s, "
                                "flops / GEMM peak) + graph build bytes / 8 TB/s, over step time"
                                if args.mode == "fwd" else
                                "sum over the training step's kernels (bench.train_step_dataflow:"
                                " graph build + transpose, forward with alpha, BCE, attention "
                                "norm, every layer's backward, Adam) of max(unique bytes / 8 TB/s,"
                                " flops / GEMM peak), over step time"
                                if ds == "PPI" else "omitted: only the PPI step is priced"),
        "l2_gather_GBps": round(l2_gather / step_s / 1e9, 1),
        "hbm_measured": pmc_step_bytes(pm, ms, pmc_path),
        "roofline": ordered[0] if ordered else None,
        "roofline_other": ordered[1] if len(ordered) > 1 else None,
        "kernels": kernel_summary(summ, n_instr),
    }
    if replay_verified is not None:
        result["replay_verified"] = replay_verified
        result["replay_check"] = ("after the timed loop: static input replaced, static output and "
                                  "every layer's alpha poisoned with NaN outside the graph, one "
                                  "replay; " + replay_detail)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.mode == "fwd":
        result["cpu_baseline"] = cpu_baseline(model, cfg, ds, 8 if ds == "PATTERN" else 1)
    result["config"]["tuning"] = tuning_changes()
    if (rank == 0 and world == 1 and args.mode == "fwd" and ds == "PPI"
            and not args.no_train_leg):
        result.update(run_train_leg(args))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if replay_verified is False:
        raise SystemExit("bench.py: a replay of the captured step differs from an eager step ("
                         + replay_detail + ")")
    if reducer is not None:
        reducer.remove()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
