"""ORACLE — test infrastructure only. CPU restatement of the reference GATLayer, in numpy.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker / the timed CPU baseline. The product path (`gat-pytorch_amd/gatx`)
never imports it and fails loudly when its HIP library is missing.

What it restates (reference = loodvn/gat-pytorch, `/root/reference`, read as text):
  * `add_remaining_self_loops` / `maybe_num_nodes`  — `models/utils.py:47-72`
  * `sum_over_neighbourhood` (scatter_add_ by target) — `models/utils.py:6-27`
  * `GATLayer.forward`                                 — `models/gat_layer.py:42-140`
  * autograd of that forward, in closed form           — SURVEY.md §8(a) row a14
  * `GATModel.forward` / `forward_and_return_attention` wiring — `models/GATModel.py:120-187`
  * `GATModel.calc_attention_norm`                     — `models/GATModel.py:189-234`
It keeps the reference's dataflow on purpose (materialised per-edge gathers, the concatenated
(E, NH*2F) attention pairs multiplied by `a`, scatter-adds), because it doubles as the "port" CPU
baseline timed by bench.py.

Parity pinning: `tests/golden/*.npz` hold outputs of the reference itself, imported in the build
container by `tests/golden/make_goldens.py`; `tests/test_oracle_golden.py` checks this module
against every one of them (forward, returned edge_index / alpha, and all gradients).

The dropout mask is the product kernel's counter-based hash (`dropout_keep`), restated here so a
train-mode forward/backward can be reproduced exactly; the reference's own `nn.Dropout` draws from
torch's global RNG, which no other implementation can match bit for bit.
"""
from __future__ import annotations

import numpy as np

LEAKY_SLOPE = 0.01   # nn.LeakyReLU() default, models/gat_layer.py:87
SOFTMAX_EPS = 1e-8   # models/gat_layer.py:109


# --------------------------------------------------------------------------- graph helpers
def maybe_num_nodes(edge_index: np.ndarray, num_nodes=None) -> int:
    """models/utils.py:70-72 — max()+1 of the whole edge_index (raises on empty, like torch)."""
    if num_nodes is not None:
        return int(num_nodes)
    if edge_index.size == 0:
        raise RuntimeError("max(): Expected reduction dim to be specified for input.numel() == 0")
    return int(edge_index.max()) + 1


def add_remaining_self_loops(edge_index: np.ndarray, num_nodes=None) -> np.ndarray:
    """models/utils.py:47-67 — drop src==dst edges, append (i, i) for i < max+1, keep order."""
    N = maybe_num_nodes(edge_index, num_nodes)
    row, col = edge_index[0], edge_index[1]
    mask = row != col
    loops = np.arange(N, dtype=edge_index.dtype)
    return np.concatenate([edge_index[:, mask], np.stack([loops, loops])], axis=1)


def segment_sum(values: np.ndarray, index: np.ndarray, num_segments: int) -> np.ndarray:
    """`values.new_zeros(shape).scatter_add_(0, index, values)` (models/utils.py:17-20): sums of
    the rows of `values` per target id, taken in edge order (stable sort + reduceat)."""
    out = np.zeros((num_segments,) + values.shape[1:], dtype=values.dtype)
    if values.shape[0] == 0:
        return out
    if index.min() < 0 or index.max() >= num_segments:
        raise IndexError("index out of bounds in scatter_add_")
    order = np.argsort(index, kind="stable")
    idx_sorted = index[order]
    starts = np.flatnonzero(np.r_[True, idx_sorted[1:] != idx_sorted[:-1]])
    sums = np.add.reduceat(values[order], starts, axis=0)
    out[idx_sorted[starts]] = sums
    return out


# --------------------------------------------------------------------------- dropout hash
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def dropout_keep(seed: int, num_edges: int, num_heads: int, p: float) -> np.ndarray:
    """Keep-mask (E', NH) bool of the HIP kernels' attention dropout (restated from
    gat-pytorch_amd/csrc/gatx_common.h `dropout_keep`): element (e, h) of the returned-order
    alpha is kept iff u >= p, u = top-24 bits of splitmix64(seed + (e*NH + h + 1)*gamma) / 2^24."""
    with np.errstate(over="ignore"):
        k = np.arange(1, num_edges * num_heads + 1, dtype=np.uint64)
        z = np.uint64(seed & ((1 << 64) - 1)) + k * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return (u >= np.float32(p)).reshape(num_edges, num_heads)


# --------------------------------------------------------------------------- layer
def gat_layer_forward(x, edge_index, W, a, num_heads, out_features, concat, bias=None,
                      add_self_loops=True, const_attention=False, dropout_p=0.0, keep=None,
                      dtype=np.float32):
    """GATLayer.forward (models/gat_layer.py:42-140), eval or train with an explicit keep-mask.

    x (N, F_in); edge_index (2, E) int; W (NH*F, F_in) = `W.weight`; a (NH, NH*2F) = `a.weight`
    (ignored when const_attention); bias (NH*F,) = `bias_param` or None; keep (E', NH) bool or
    None (no dropout). Returns (out, edge_index', alpha, cache)."""
    x = np.asarray(x, dtype=dtype)
    W = np.asarray(W, dtype=dtype)
    NH, F = num_heads, out_features
    if add_self_loops:                                                      # :53-54
        edge_index = add_remaining_self_loops(edge_index)
    N = x.shape[0]                                                          # :56
    E = edge_index.shape[1]                                                 # :57
    src, dst = edge_index[0].astype(np.int64), edge_index[1].astype(np.int64)   # :59
    if E and (src.max() >= N or dst.max() >= N or min(src.min(), dst.min()) < -N):
        raise IndexError("edge_index out of range for x")
    Wh = (x @ W.T).reshape(N, NH, F)                                        # :64-65
    Wh_src = Wh[src]                                                        # :70
    Wh_dst = Wh[dst]                                                        # :71
    cache = dict(x=x, W=W, src=src, dst=dst, N=N, NH=NH, F=F, concat=concat,
                 const_attention=const_attention, Wh=Wh, dtype=dtype)
    if not const_attention:
        a = np.asarray(a, dtype=dtype)
        pairs = np.concatenate([Wh_src, Wh_dst], axis=-1).reshape(E, NH * 2 * F)   # :76-81
        raw = pairs @ a.T                                                   # :82
        M = raw.max()                                                       # :85
        shifted = raw - M
        t = np.where(shifted > 0, shifted, shifted * dtype(LEAKY_SLOPE))    # :87
        cache.update(a=a, pairs=pairs, raw=raw, M=M)
    else:
        t = np.zeros((E, NH), dtype=dtype)                                  # :92
    ex = np.exp(t)                                                          # :96
    den = segment_sum(ex, dst, N)                                           # :99-103
    den_b = den[dst]                                                        # :106
    alpha = ex / (den_b + dtype(SOFTMAX_EPS))                               # :109
    if keep is not None and dropout_p > 0:                                  # :113-115
        scale = keep.astype(dtype) / dtype(1.0 - dropout_p)
        alpha_d = alpha * scale
    else:
        scale = None
        alpha_d = alpha
    msg = alpha_d.reshape(E, NH, 1) * Wh_src                                # :119
    out = segment_sum(msg, dst, N)                                          # :123-127
    if concat:                                                              # :129-132
        out = out.reshape(N, NH * F)
    else:
        out = out.mean(axis=1)
    if bias is not None:                                                    # :134-135
        out = out + np.asarray(bias, dtype=dtype)
    cache.update(ex=ex, den=den, alpha=alpha, alpha_d=alpha_d, scale=scale,
                 edge_index=edge_index, bias=bias)
    return out, edge_index, alpha, cache


def gat_layer_backward(cache, g_out, g_alpha=None):
    """Gradients of gat_layer_forward's (out, alpha) w.r.t. (x, W, a, bias): the closed form of
    torch autograd through models/gat_layer.py:64-135, keeping the
    reference's dataflow (gather backward = scatter, cat/linear backward through `pairs`).
    `max()` splits its gradient evenly over ties, as torch's full-reduction max does."""
    dt = cache["dtype"]
    N, NH, F = cache["N"], cache["NH"], cache["F"]
    src, dst, Wh, x, W = cache["src"], cache["dst"], cache["Wh"], cache["x"], cache["W"]
    E = src.shape[0]
    g_out = np.asarray(g_out, dtype=dt)
    g_bias = g_out.sum(axis=0) if cache["bias"] is not None else None
    if cache["concat"]:
        go = g_out.reshape(N, NH, F)
    else:
        go = np.broadcast_to(g_out[:, None, :] / dt(NH), (N, NH, F))
    go_dst = go[dst]                                                        # backward of scatter
    Wh_src = Wh[src]
    g_alpha_d = np.einsum("ehf,ehf->eh", go_dst, Wh_src)                    # backward of :119
    g_Wh = segment_sum(cache["alpha_d"][:, :, None] * go_dst, src, N)
    g_a = None
    if not cache["const_attention"]:
        ga = g_alpha_d * cache["scale"] if cache["scale"] is not None else g_alpha_d
        if g_alpha is not None:
            ga = ga + np.asarray(g_alpha, dtype=dt)
        alpha, ex, den = cache["alpha"], cache["ex"], cache["den"]
        c = segment_sum(ga * alpha, dst, N)                                 # softmax backward
        g_ex = (ga - c[dst]) / (den[dst] + dt(SOFTMAX_EPS))
        g_t = g_ex * ex                                                     # exp backward
        raw, M = cache["raw"], cache["M"]
        g_shift = np.where(raw - M > 0, g_t, g_t * dt(LEAKY_SLOPE))         # leaky_relu backward
        ties = raw == M
        g_raw = g_shift + ties * (-g_shift.sum() / dt(ties.sum()))          # max() backward
        g_a = g_raw.T @ cache["pairs"]                                      # linear backward
        g_pairs = (g_raw @ cache["a"]).reshape(E, NH, 2 * F)
        g_Wh = g_Wh + segment_sum(g_pairs[:, :, :F], src, N) + segment_sum(g_pairs[:, :, F:], dst, N)
    g_Wh = g_Wh.reshape(N, NH * F)
    g_W = g_Wh.T @ x
    g_x = g_Wh @ W
    return dict(x=g_x, W=g_W, a=g_a, bias=g_bias)


# --------------------------------------------------------------------------- model wiring
def elu(v):
    return np.where(v > 0, v, np.expm1(np.minimum(v, 0))).astype(v.dtype)


def gat_model_forward(x, edge_index, layers, skips, num_heads, out_features, concat, add_skip,
                      dtype=np.float32):
    """GATModel.forward_and_return_attention in eval mode (models/GATModel.py:153-187): per layer
    GATLayer(add_self_loops=True, bias=False) -> skip (concat add, or head-mean add) -> ELU except
    after the last layer. `layers[i]` = (W, a); `skips` = list of skip weights (None = Identity)
    for the layers with add_skip[i]. Returns (out, edge_index', [alpha_i])."""
    x = np.asarray(x, dtype=dtype)
    L = len(layers)
    alphas, skip_i = [], 0
    for i in range(L):
        inp = x
        W, a = layers[i]
        x, edge_index, alpha, _ = gat_layer_forward(x, edge_index, W, a, num_heads[i],
                                                    out_features[i], concat[i], dtype=dtype)
        alphas.append(alpha)
        if add_skip[i]:
            Ws = skips[skip_i]
            skip_i += 1
            so = inp if Ws is None else inp @ np.asarray(Ws, dtype=dtype).T
            if concat[i]:
                x = x + so
            else:
                x = x + so.reshape(-1, num_heads[i], out_features[i]).mean(axis=1)
        if i != L - 1:
            x = elu(x)
    return x, edge_index, alphas


def calc_attention_norm(edge_index, attention_list):
    """models/GATModel.py:189-234: mean over layers of ||alpha * in_degree[dst] - 1||_1 / E."""
    dst = edge_index[1].astype(np.int64)
    E = dst.shape[0]
    first = attention_list[0]
    deg = segment_sum(np.ones(E, dtype=first.dtype), dst, E)[dst]   # aggregated_shape=(E,)
    tot = 0.0
    for al in attention_list:
        tot = tot + np.abs(al * deg[:, None] - 1.0).sum() / E
    return tot / len(attention_list)


def calc_attention_norm_grad(edge_index, attention_list, g=1.0):
    """Gradient of calc_attention_norm w.r.t. each alpha: g * sgn(alpha*deg - 1) * deg / (E*L)
    (torch's d|x|/dx = sgn x, 0 at 0)."""
    dst = edge_index[1].astype(np.int64)
    E = dst.shape[0]
    deg = segment_sum(np.ones(E, dtype=np.float64), dst, E)[dst]
    L = len(attention_list)
    out = []
    for al in attention_list:
        d = deg.astype(al.dtype)[:, None]
        t = al * d - al.dtype.type(1.0)   # in alpha's precision, like the reference's fp32
        out.append(g * np.sign(t).astype(np.float64) * deg[:, None] / (E * L))
    return out


def gat_model_forward_backward(x, edge_index, layers, skips, num_heads, out_features, concat,
                               add_skip, g_out, dtype=np.float64, g_alphas=None):
    """gat_model_forward plus its backward for an upstream gradient g_out: the layer backward
    (gat_layer_backward) chained through ELU (d elu = 1 for x > 0 else exp(x)), the skip add
    (concat: add; head-mean: add of the skip's per-head mean, models/GATModel.py:135-145) and
    the skip projection. g_alphas: optional per-layer upstream gradients of the returned alphas
    (a loss on the attention, e.g. calc_attention_norm). g_out may be a callable out -> g_out
    (a loss of the forward's output). Returns (out, {"W": [...], "a": [...], "skip": [...],
    "x": g_x})."""
    x = np.asarray(x, dtype=dtype)
    L = len(layers)
    saved, skip_i = [], 0
    for i in range(L):
        inp = x
        W, a = layers[i]
        o, edge_index, alpha, cache = gat_layer_forward(x, edge_index, W, a, num_heads[i],
                                                        out_features[i], concat[i], dtype=dtype)
        Ws = None
        if add_skip[i]:
            Ws = skips[skip_i]
            skip_i += 1
            so = inp if Ws is None else inp @ np.asarray(Ws, dtype=dtype).T
            o = o + (so if concat[i] else so.reshape(-1, num_heads[i], out_features[i]).mean(axis=1))
        saved.append((inp, cache, o, Ws))
        x = elu(o) if i != L - 1 else o
    g = np.asarray(g_out(x) if callable(g_out) else g_out, dtype=dtype)
    gW, ga, gs = [None] * L, [None] * L, []
    for i in reversed(range(L)):
        inp, cache, pre, Ws = saved[i]
        g_pre = g * np.where(pre > 0, 1.0, np.exp(np.minimum(pre, 0))) if i != L - 1 else g
        gr = gat_layer_backward(cache, g_pre, None if g_alphas is None else g_alphas[i])
        gW[i], ga[i] = gr["W"], gr["a"]
        g_inp = gr["x"]
        if add_skip[i]:
            if concat[i]:
                g_so = g_pre
            else:
                g_so = np.repeat(g_pre[:, None, :] / num_heads[i], num_heads[i], axis=1)
                g_so = g_so.reshape(g_pre.shape[0], -1)
            if Ws is None:
                g_inp = g_inp + g_so
                gs.append(None)
            else:
                Wsd = np.asarray(Ws, dtype=dtype)
                gs.append(g_so.T @ inp)
                g_inp = g_inp + g_so @ Wsd
        g = g_inp
    return x, {"W": gW, "a": ga, "skip": gs[::-1], "x": g}


# --------------------------------------------------------------------------- task module step
def cross_entropy_grad(logits, labels, rows):
    """d/d logits of torch.nn.CrossEntropyLoss(reduction='mean')(logits[rows], labels[rows])
    (models/planetoid_gat.py:11,28): (softmax - onehot) / |rows| on the masked rows, 0 elsewhere.
    Returns (loss, grad)."""
    z = logits[rows].astype(np.float64)
    z = z - z.max(axis=1, keepdims=True)
    p = np.exp(z)
    p /= p.sum(axis=1, keepdims=True)
    n = len(rows)
    y = labels[rows]
    loss = -np.log(p[np.arange(n), y]).mean()
    g = np.zeros(logits.shape, dtype=np.float64)
    p[np.arange(n), y] -= 1.0
    g[rows] = p / n
    return loss, g


def planetoid_step_grads(x, edge_index, layers, num_heads, out_features, concat, labels, rows,
                         attention_reward):
    """PlanetoidGAT.training_step's gradients (`models/planetoid_gat.py:15-30`) in eval-mode
    arithmetic (no dropout): loss = CE(out[train], y[train]) + attention_reward *
    calc_attention_norm(edge_index', alphas). Returns (loss, grads) with grads as
    gat_model_forward_backward's."""
    L = len(layers)
    out, ei2, alphas = gat_model_forward(x, edge_index, layers, [], num_heads, out_features,
                                         concat, [False] * L, dtype=np.float64)
    ce, g_out = cross_entropy_grad(out, labels, rows)
    norm = calc_attention_norm(ei2, alphas)
    g_al = [attention_reward * g for g in calc_attention_norm_grad(ei2, alphas)]
    _, grads = gat_model_forward_backward(x, edge_index, layers, [], num_heads, out_features,
                                          concat, [False] * L, g_out, g_alphas=g_al)
    return ce + attention_reward * norm, grads


def bce_logits_grad(logits, target, pos_weight=None):
    """torch.nn.BCEWithLogitsLoss(reduction='mean', pos_weight=p) and its gradient
    (`models/ppi_gat.py:11,19`; PatternGAT's class-balanced form, `models/pattern_gat.py:11-15,
    23`): l = -(p y log s(x) + (1 - y) log(1 - s(x))), mean over every element;
    d l / d x = ((p y + 1 - y) s(x) - p y) / n. Returns (loss, grad)."""
    x = np.asarray(logits, dtype=np.float64)
    y = np.asarray(target, dtype=np.float64)
    p = 1.0 if pos_weight is None else float(pos_weight)
    # log s(x) = -softplus(-x), log(1 - s(x)) = -softplus(x), stably
    sp_pos = np.logaddexp(0.0, x)
    sp_neg = np.logaddexp(0.0, -x)
    n = x.size
    loss = float((p * y * sp_neg + (1.0 - y) * sp_pos).sum() / n)
    s = 1.0 / (1.0 + np.exp(-x))
    return loss, ((p * y + 1.0 - y) * s - p * y) / n


def model_step_grads(task, x, edge_index, layers, skips, num_heads, out_features, concat,
                     add_skip, labels, rows, coef):
    """One task module's training-step loss and gradients in fp64 (no dropout):
    * "planetoid": PlanetoidGAT.training_step (`models/planetoid_gat.py:15-30`) = CE(out[rows],
      y[rows]) + coef * calc_attention_norm;
    * "ppi": PPI_GAT.training_step (`models/ppi_gat.py:15-33`) = BCEWithLogits(out, y), plus
      coef * calc_attention_norm only when coef != 0 (`:28-29`);
    * "pattern": PatternGAT.training_step (`models/pattern_gat.py:18-25`) = BCEWithLogits(
      squeeze(out), y, pos_weight = 1 / 0.1765).
    Returns (loss, grads) with grads as gat_model_forward_backward's."""
    out, ei2, alphas = gat_model_forward(x, edge_index, layers, skips, num_heads, out_features,
                                         concat, add_skip, dtype=np.float64)
    if task == "planetoid":
        loss, g_out = cross_entropy_grad(out, labels, rows)
    elif task == "ppi":
        loss, g_out = bce_logits_grad(out, labels)
    else:
        loss, g = bce_logits_grad(out[:, 0], labels, pos_weight=1 / 0.1765)
        g_out = g[:, None]
    g_al = None
    if coef != 0.0 and task != "pattern":
        loss = loss + coef * calc_attention_norm(ei2, alphas)
        g_al = [coef * g for g in calc_attention_norm_grad(ei2, alphas)]
    _, grads = gat_model_forward_backward(x, edge_index, layers, skips, num_heads, out_features,
                                          concat, add_skip, g_out, g_alphas=g_al)
    return loss, grads
