"""Generate the golden fixtures in tests/golden/ by running the REFERENCE GATLayer itself.

Runs only in the build container, where /root/reference exists and imports (the
hot path `models/gat_layer.py` + `models/utils.py` need only torch). Nothing here ships to the GPU
box; the fixtures it writes are data (inputs that are too big to store are regenerated from
splitmix64 seeds by gatx.data; expected outputs and gradients are stored).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py
    (--steps: only the round-5 training-step goldens, step_cases)

For each case: build inputs, run `GATLayer.forward(x, edge_index, return_attention_weights=True)`
in fp32 (torch CPU), then backprop loss = <out, g_out> + <alpha, g_alpha> with torch autograd and
store out, edge_index', alpha and the gradients of x, W.weight, a.weight, bias_param. Large gradient
arrays are stored as a row sample plus whole-array checksums (sum, sum|.|, sum of squares).
Model-level cases wire reference GATLayers exactly as GATModel.forward_and_return_attention does
(`models/GATModel.py:153-187`), since GATModel itself needs pytorch_lightning, which is absent.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "gat-pytorch_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

from models.gat_layer import GATLayer  # noqa: E402  (the reference)
from models.utils import explicit_broadcast, sum_over_neighbourhood  # noqa: E402  (the reference)
from gatx import data as gdata  # noqa: E402
from gatx.checkpoint import read_state_dict  # noqa: E402
from oracle.gat_oracle import dropout_keep  # noqa: E402

CKPT = "/root/reference/checkpoints"
BIG = 200_000  # arrays with more elements are stored as sample + checksums


def checksums(a: np.ndarray) -> np.ndarray:
    a = a.astype(np.float64)
    return np.array([a.sum(), np.abs(a).sum(), (a * a).sum(), np.abs(a).max()])


def sample_rows(n_rows: int, k: int = 48) -> np.ndarray:
    rows = np.unique(np.r_[np.arange(min(8, n_rows)), gdata.randint(99, k, n_rows)])
    return rows.astype(np.int64)


def put(store: dict, name: str, arr: np.ndarray):
    arr = np.asarray(arr)
    if arr.size > BIG:
        rows = sample_rows(arr.shape[0])
        store[f"{name}__rows"] = rows
        store[f"{name}__sample"] = arr[rows]
        store[f"{name}__checksums"] = checksums(arr)
    else:
        store[name] = arr


def ref_layer(in_f, F, NH, concat, W, a, bias=None, add_loops=True, const=False, dropout=0.0):
    layer = GATLayer(in_f, F, NH, concat, dropout=dropout, add_self_loops=add_loops,
                     bias=bias is not None, const_attention=const)
    with torch.no_grad():
        layer.W.weight.copy_(torch.from_numpy(W))
        if not const:
            layer.a.weight.copy_(torch.from_numpy(a))
        if bias is not None:
            layer.bias_param.copy_(torch.from_numpy(bias))
    return layer


def run_layer_case(name, x, edge_index, in_f, F, NH, concat, W, a, bias=None, add_loops=True,
                   const=False, dropout=0.0, seed=0, gen=None, store_x=None, wgen=None):
    layer = ref_layer(in_f, F, NH, concat, W, a, bias, add_loops, const, dropout)
    if dropout > 0:
        # train-mode dropout with the HIP kernels' counter-based mask
        def injected(t):
            keep = dropout_keep(seed, t.shape[0], t.shape[1], dropout)
            return t * torch.from_numpy(keep.astype(np.float32)) / (1.0 - dropout)
        layer._modules.pop("dropout_layer", None)
        object.__setattr__(layer, "dropout_layer", injected)
    xt = torch.from_numpy(x).requires_grad_(True)
    et = torch.from_numpy(edge_index)
    out, (ei2, alpha) = layer(xt, et, return_attention_weights=True)
    grads_note = None
    if edge_index.dtype == np.int32:
        # torch 2.10 CPU: the backward of scatter_add_ with an int32 (expanded) index returns
        # wrong gradients (probed: |d| up to 45 on a 10x3 toy), while the forward is exact.
        # Forward goldens come from the int32 run; gradients from the same inputs as int64.
        grads_note = "gradients from the int64 copy of edge_index (torch int32 scatter_add_ bwd bug)"
        xt = torch.from_numpy(x).requires_grad_(True)
        out, (_, alpha) = layer(xt, torch.from_numpy(edge_index.astype(np.int64)),
                                return_attention_weights=True)
    g_out = gdata.normal(7, out.numel()).reshape(tuple(out.shape))
    g_alpha = 0.1 * gdata.normal(8, alpha.numel()).reshape(tuple(alpha.shape))
    loss = (out * torch.from_numpy(g_out)).sum()
    if not const:
        loss = loss + (alpha * torch.from_numpy(g_alpha)).sum()
    loss.backward()
    store = {}
    meta = dict(kind="layer", in_features=in_f, out_features=F, num_heads=NH, concat=concat,
                add_self_loops=add_loops, const_attention=const, dropout=dropout, seed=seed,
                has_bias=bias is not None, edge_dtype=str(edge_index.dtype), gen=gen,
                use_g_alpha=not const, wgen=wgen, grads_note=grads_note)
    if gen is None or store_x:
        put(store, "x", x)
        store["edge_index"] = edge_index
    if wgen is None:      # trained / hand-made weights are stored; xavier ones regenerate
        store["W"] = W
        if not const:
            store["a"] = a
    if bias is not None:
        store["bias"] = bias
    put(store, "out", out.detach().numpy())
    store["edge_index_out"] = ei2.numpy().astype(np.int64)
    put(store, "alpha", alpha.detach().numpy())
    put(store, "grad_x", xt.grad.numpy())
    put(store, "grad_W", layer.W.weight.grad.numpy())
    if not const:
        put(store, "grad_a", layer.a.weight.grad.numpy())
    if bias is not None:
        put(store, "grad_bias", layer.bias_param.grad.numpy())
    store["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **store)
    print(f"{name}: N={x.shape[0]} E'={ei2.shape[1]} out={tuple(out.shape)}")


def gen_batch(gen):
    b = gdata.uniform_graph_batch(gen["G"], gen["n"], gen["e"], gen["in_features"],
                                  graph_seed=gen.get("graph_seed", 42),
                                  feature_seed=gen.get("feature_seed", 1),
                                  features=gen.get("features", "normal"))
    return b.x, b.edge_index


def ref_attention_norm(edge_index, alphas):
    """GATModel.calc_attention_norm (`models/GATModel.py:189-230`, logging removed) on the
    reference's own helpers; returns the value and d value / d alpha_l for an upstream 1."""
    att = [torch.from_numpy(a).requires_grad_(True) for a in alphas]
    nb = edge_index[1]
    first = att[0]
    degrees = sum_over_neighbourhood(torch.ones_like(first[:, 0]), neighbourhood_indices=nb,
                                     aggregated_shape=first[:, 0].size(), broadcast_back=True)
    norm = torch.tensor(0.0)
    for a in att:
        tmp = explicit_broadcast(degrees, a)
        norm = norm + torch.norm(a * tmp - 1.0, p=1) / nb.size(0)
    norm = norm / torch.tensor(len(att))
    norm.backward()
    return norm.detach().numpy(), [a.grad.numpy() for a in att]


def main(models_only=False):
    torch.set_num_threads(8)
    sd_cora = read_state_dict(f"{CKPT}/Cora-100epochs.ckpt")
    sd_pat = read_state_dict(f"{CKPT}/PATTERN-100epochs.ckpt")
    if models_only:
        return model_cases(sd_pat)

    # 1-3: Cora shapes (SURVEY.md §8c goldens 1-2), trained and xavier weights
    gen = dict(G=1, n=2708, e=10556, in_features=1433, features="bernoulli")
    x, ei = gen_batch(gen)
    run_layer_case("cora_l0_trained", x, ei, 1433, 8, 8, True,
                   sd_cora["gat_layer_list.0.W.weight"], sd_cora["gat_layer_list.0.a.weight"],
                   gen=gen)
    run_layer_case("cora_l0_xavier", x, ei, 1433, 8, 8, True,
                   gdata.xavier_uniform(0, 64, 1433), gdata.xavier_uniform(1, 8, 128), gen=gen,
                   wgen=[0, 1])
    gen1 = dict(G=1, n=2708, e=10556, in_features=64)
    x1, ei1 = gen_batch(gen1)
    run_layer_case("cora_l1_mean_trained", x1, ei1, 64, 7, 1, False,
                   sd_cora["gat_layer_list.1.W.weight"], sd_cora["gat_layer_list.1.a.weight"],
                   gen=gen1)

    # 4: PPI layer shapes on a reduced single graph (golden 3, shrunk so fixtures stay small)
    for lname, (fin, F, NH, cc) in {"l0": (50, 256, 4, True), "l1": (1024, 256, 4, True),
                                     "l2": (1024, 121, 6, False)}.items():
        g = dict(G=1, n=256, e=7000, in_features=fin, feature_seed=11)
        xx, ee = gen_batch(g)
        run_layer_case(f"ppi_small_{lname}", xx, ee, fin, F, NH, cc,
                       gdata.xavier_uniform(20, NH * F, fin),
                       gdata.xavier_uniform(21, NH, NH * 2 * F), gen=g, wgen=[20, 21])

    # 5: adversarial logits: a x 1e3 (segment alpha-sums << 1, |g_M| large)
    g = dict(G=2, n=100, e=1500, in_features=16, feature_seed=12)
    xx, ee = gen_batch(g)
    run_layer_case("adversarial_a1e3", xx, ee, 16, 8, 4, True, gdata.xavier_uniform(30, 32, 16),
                   1e3 * gdata.xavier_uniform(31, 4, 64), gen=g, store_x=True)

    # 6: edge cases (all stored in full)
    rng_x = lambda n, f, s: gdata.normal(s, n * f).reshape(n, f)
    # trailing isolated nodes: x has 60 rows, edges touch only 0..49 -> rows 50.. output 0
    ei = np.stack([gdata.randint(40, 300, 50), gdata.randint(41, 300, 50)])
    run_layer_case("edge_trailing_isolated", rng_x(60, 12, 42), ei, 12, 5, 3, True,
                   gdata.xavier_uniform(42, 15, 12), gdata.xavier_uniform(43, 3, 30))
    # pre-existing self-loops and duplicate edges
    ei = np.stack([gdata.randint(44, 200, 40), gdata.randint(45, 200, 40)])
    ei = np.concatenate([ei, ei[:, :30], np.stack([np.arange(0, 40, 3)] * 2)], axis=1)
    run_layer_case("edge_selfloops_duplicates", rng_x(40, 10, 46), ei, 10, 6, 2, True,
                   gdata.xavier_uniform(47, 12, 10), gdata.xavier_uniform(48, 2, 24))
    # const attention (no `a`), mean heads
    ei = np.stack([gdata.randint(50, 500, 64), gdata.randint(51, 500, 64)])
    run_layer_case("edge_const_attention", rng_x(64, 9, 52), ei, 9, 4, 3, False,
                   gdata.xavier_uniform(53, 12, 9), None, const=True)
    # bias (nonzero), concat
    run_layer_case("edge_bias", rng_x(64, 9, 54), ei, 9, 4, 3, True,
                   gdata.xavier_uniform(55, 12, 9), gdata.xavier_uniform(56, 3, 24),
                   bias=gdata.normal(57, 12))
    # bias with mean heads (bias has NH*F entries but the output only F: reference would fail)
    # int32 edge_index
    run_layer_case("edge_int32_index", rng_x(64, 9, 58), ei.astype(np.int32), 9, 4, 3, True,
                   gdata.xavier_uniform(59, 12, 9), gdata.xavier_uniform(60, 3, 24))
    # no self loops added, zero in-degree nodes present, self loops in input kept
    ei = np.stack([gdata.randint(61, 90, 64), gdata.randint(62, 90, 32)])
    ei = np.concatenate([ei, np.array([[5, 7], [5, 7]])], axis=1)
    run_layer_case("edge_no_selfloops", rng_x(64, 9, 63), ei, 9, 4, 3, True,
                   gdata.xavier_uniform(64, 12, 9), gdata.xavier_uniform(65, 3, 24),
                   add_loops=False)
    # dropout 0.6 (Cora's rate) with the kernel's hash mask
    ei = np.stack([gdata.randint(66, 600, 80), gdata.randint(67, 600, 80)])
    run_layer_case("edge_dropout", rng_x(80, 11, 68), ei, 11, 8, 8, True,
                   gdata.xavier_uniform(69, 64, 11), gdata.xavier_uniform(70, 8, 128),
                   dropout=0.6, seed=1234)
    # all logits tied (a = 0): max() gradient split over every entry
    run_layer_case("edge_ties_a_zero", rng_x(80, 11, 71), ei, 11, 8, 2, True,
                   gdata.xavier_uniform(72, 16, 11), np.zeros((2, 32), np.float32))
    # tiny graphs: a single edge, a single node
    run_layer_case("edge_single_edge", rng_x(3, 4, 73), np.array([[0], [2]]), 4, 3, 2, True,
                   gdata.xavier_uniform(74, 6, 4), gdata.xavier_uniform(75, 2, 12))
    run_layer_case("edge_single_node", rng_x(1, 4, 76), np.array([[0], [0]]), 4, 3, 2, False,
                   gdata.xavier_uniform(77, 6, 4), gdata.xavier_uniform(78, 2, 12))
    # F not a multiple of 4, odd head count (exercises padding), concat
    ei = np.stack([gdata.randint(79, 700, 70), gdata.randint(80, 700, 70)])
    run_layer_case("edge_odd_widths", rng_x(70, 13, 81), ei, 13, 7, 5, True,
                   gdata.xavier_uniform(82, 35, 13), gdata.xavier_uniform(83, 5, 70))

    extra_cases()
    model_cases(sd_pat)


def extra_cases():
    """Round-2 additions: head-mean layers with more than 8 heads (gat_layer.py:132 accepts any
    NH; the HIP path runs them as head groups accumulated in stream order), and the Citeseer /
    Pubmed trained checkpoints (data_utils.py:36-47) through the layer: Citeseer L0
    (3703 -> 8 x 8 concat), Pubmed L0 (500 -> 8 x 8) and Pubmed's 8-head MEAN output layer
    (64 -> 8 x 3, mean) on synthetic graphs of the datasets' sizes (PyG stats)."""
    g = dict(G=2, n=100, e=1500, in_features=24, feature_seed=17)
    xx, ee = gen_batch(g)
    run_layer_case("mean_nh12", xx, ee, 24, 16, 12, False, gdata.xavier_uniform(110, 192, 24),
                   gdata.xavier_uniform(111, 12, 12 * 32), gen=g, wgen=[110, 111])
    g = dict(G=2, n=90, e=1400, in_features=20, feature_seed=18)
    xx, ee = gen_batch(g)
    run_layer_case("mean_nh16", xx, ee, 20, 9, 16, False, gdata.xavier_uniform(112, 144, 20),
                   gdata.xavier_uniform(113, 16, 16 * 18), gen=g, wgen=[112, 113])
    sd_cs = read_state_dict(f"{CKPT}/Citeseer-100epochs.ckpt")
    sd_pm = read_state_dict(f"{CKPT}/Pubmed-100epochs.ckpt")
    gen = dict(G=1, n=3327, e=9104, in_features=3703, features="bernoulli", feature_seed=19)
    x, ei = gen_batch(gen)
    run_layer_case("citeseer_l0_trained", x, ei, 3703, 8, 8, True,
                   sd_cs["gat_layer_list.0.W.weight"], sd_cs["gat_layer_list.0.a.weight"],
                   gen=gen)
    gen = dict(G=1, n=19717, e=88648, in_features=500, feature_seed=20)
    x, ei = gen_batch(gen)
    run_layer_case("pubmed_l0_trained", x, ei, 500, 8, 8, True,
                   sd_pm["gat_layer_list.0.W.weight"], sd_pm["gat_layer_list.0.a.weight"],
                   gen=gen)
    gen = dict(G=1, n=19717, e=88648, in_features=64, feature_seed=21)
    x, ei = gen_batch(gen)
    run_layer_case("pubmed_l1_mean_trained", x, ei, 64, 3, 8, False,
                   sd_pm["gat_layer_list.1.W.weight"], sd_pm["gat_layer_list.1.a.weight"],
                   gen=gen)


def model_cases(sd_pat):
    # 7: model level — PATTERN 4 layers with trained weights (golden 4), 2 graphs
    gp = dict(G=2, n=119, e=6099, in_features=3, feature_seed=13)
    xp, ep = gen_batch(gp)
    model_case("pattern_model_trained", xp, ep, gp,
               [(sd_pat[f"gat_layer_list.{i}.W.weight"], sd_pat[f"gat_layer_list.{i}.a.weight"])
                for i in range(4)],
               [sd_pat[f"skip_layer_list.{i}.weight"] for i in range(4)], "PATTERN")
    # PPI wiring (skip identity on layer 1) on a reduced graph, xavier weights
    gq = dict(G=1, n=200, e=5000, in_features=50, feature_seed=14)
    xq, eq = gen_batch(gq)
    dims = [(50, 256, 4), (1024, 256, 4), (1024, 121, 6)]
    model_case("ppi_model_small", xq, eq, gq,
               [(gdata.xavier_uniform(90 + i, NH * F, fin),
                 gdata.xavier_uniform(95 + i, NH, NH * 2 * F)) for i, (fin, F, NH) in enumerate(dims)],
               [None], "PPI", wgen=[[90 + i, 95 + i] for i in range(3)])


def planetoid_model_cases():
    """Round-4 additions (BASELINE configs 1-2 at model level): the 2-layer Cora / Citeseer /
    Pubmed GATModels with their TRAINED checkpoints (`checkpoints/*-100epochs.ckpt`) in eval
    mode — output logits, both layers' alphas, calc_attention_norm and its gradient — on
    synthetic graphs of the datasets' sizes (the layer cases' graphs)."""
    for ds, gen in (("Cora", dict(G=1, n=2708, e=10556, in_features=1433, features="bernoulli")),
                    ("Citeseer", dict(G=1, n=3327, e=9104, in_features=3703,
                                      features="bernoulli", feature_seed=19)),
                    ("Pubmed", dict(G=1, n=19717, e=88648, in_features=500, feature_seed=20))):
        sd = read_state_dict(f"{CKPT}/{ds}-100epochs.ckpt")
        x, ei = gen_batch(gen)
        model_case(f"{ds.lower()}_model_trained", x, ei, gen,
                   [(sd[f"gat_layer_list.{i}.W.weight"], sd[f"gat_layer_list.{i}.a.weight"])
                    for i in range(2)], [], ds)


def model_case(name, x, ei, gen, layers, skips, dataset, wgen=None):
    sys.path.insert(0, REPO)
    from gatx.config import data_config
    cfg = data_config[dataset]
    heads = [1] + cfg["num_heads_per_layer"]
    widths = cfg["head_output_features_per_layer"]
    concat = cfg["heads_concat_per_layer"]
    add_skip = cfg["add_skip_connection"]
    L = cfg["num_layers"]
    mods = []
    for i in range(L):
        W, a = layers[i]
        mods.append(ref_layer(heads[i] * widths[i], widths[i + 1], heads[i + 1], concat[i], W, a))
    xt = torch.from_numpy(x)
    edge_index = torch.from_numpy(ei)
    alphas, skip_i = [], 0
    with torch.no_grad():
        for i in range(L):       # models/GATModel.py:160-185, eval mode (dropout is identity)
            layer_input = xt
            xt, (edge_index, att) = mods[i](xt, edge_index, return_attention_weights=True)
            alphas.append(att.numpy())
            if add_skip[i]:
                Ws = skips[skip_i]
                skip_i += 1
                so = layer_input if Ws is None else layer_input @ torch.from_numpy(Ws).T
                if concat[i]:
                    xt = xt + so
                else:
                    xt = xt + so.view(-1, heads[i + 1], widths[i + 1]).mean(dim=1)
            if i != L - 1:
                xt = torch.nn.functional.elu(xt)
    store = {"meta": np.array(json.dumps(dict(kind="model", dataset=dataset, gen=gen,
                                              wgen=wgen))),
             "edge_index_out": edge_index.numpy()}
    for i, (W, a) in enumerate(layers):
        if wgen is None:
            store[f"W{i}"] = W
            store[f"a{i}"] = a
    for i, s in enumerate(skips):
        if s is not None:
            store[f"skip{i}"] = s
    put(store, "out", xt.numpy())
    for i, al in enumerate(alphas):
        put(store, f"alpha{i}", al)
    # calc_attention_norm over the returned edge_index' and alphas (+ its gradient, upstream 1)
    norm, grads = ref_attention_norm(edge_index, alphas)
    store["attention_norm"] = norm
    for i, g in enumerate(grads):
        put(store, f"attention_norm_grad{i}", g)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **store)
    print(f"{name}: N={x.shape[0]} out={tuple(xt.shape)}")


def ppi_full_cases():
    """The three PPI layer shapes on one full-size PPI graph (2245 nodes, 61318 edges: SURVEY.md
    §8c golden 3 at the dataset's size, `run_config.py:18-33`); large arrays as row samples plus
    whole-array checksums."""
    for lname, (fin, F, NH, cc) in {"l0": (50, 256, 4, True), "l1": (1024, 256, 4, True),
                                     "l2": (1024, 121, 6, False)}.items():
        g = dict(G=1, n=2245, e=61318, in_features=fin, feature_seed=13)
        xx, ee = gen_batch(g)
        run_layer_case(f"ppi_full_{lname}", xx, ee, fin, F, NH, cc,
                       gdata.xavier_uniform(22, NH * F, fin),
                       gdata.xavier_uniform(23, NH, NH * 2 * F), gen=g, wgen=[22, 23])


def ref_attention_norm_graph(edge_index, att_list):
    """GATModel.calc_attention_norm (`models/GATModel.py:189-230`, logging removed) on the
    reference's own helpers, kept in the autograd graph of the alphas (a training step's loss)."""
    nb = edge_index[1]
    first = att_list[0]
    degrees = sum_over_neighbourhood(torch.ones_like(first[:, 0]), neighbourhood_indices=nb,
                                     aggregated_shape=first[:, 0].size(), broadcast_back=True)
    norm = torch.tensor(0.0)
    for a in att_list:
        tmp = explicit_broadcast(degrees, a)
        norm = norm + torch.norm(a * tmp - 1.0, p=1) / nb.size(0)
    return norm / torch.tensor(len(att_list))


def step_labels(task, N, C):
    """The synthetic labels of the step goldens (regenerated by tests/golden_io.step_labels)."""
    if task == "planetoid":
        return (gdata.randint(123, N, 1 << 30) % C).astype(np.int64), np.arange(20 * C)
    if task == "ppi":
        return gdata.randint(124, N * C, 2).reshape(N, C).astype(np.float32), None
    return gdata.randint(125, N, 2).astype(np.float32), None      # PATTERN: one logit per node


def step_case(name, base, variants):
    """Round-5: a whole task-module TRAINING STEP through reference GATLayers
    under autograd, wired as GATModel.forward_and_return_attention (`models/GATModel.py:153-187`;
    `forward`, `:120-151`, for PATTERN: the same layers and skips), with the task's loss:
    * PlanetoidGAT.training_step (`models/planetoid_gat.py:15-30`): CrossEntropy over the train
      rows + attention_reward x calc_attention_norm;
    * PPI_GAT.training_step (`models/ppi_gat.py:15-33`): BCEWithLogits (mean) + the norm x
      attention_penalty, added only when the penalty is non-zero;
    * PatternGAT.training_step (`models/pattern_gat.py:18-25`): squeeze, BCEWithLogits with
      pos_weight 1 / 0.1765.
    Model dropout is 0 (the Planetoid configs' 0.6 draws torch's RNG, which no kernel can
    reproduce; the layer goldens pin the dropout path with an injected mask). `base` names the
    model golden whose inputs and weights the step uses; stored per variant (the reward /
    penalty): the loss and the gradients of every W, a and Linear skip weight."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from golden_io import load_model_case
    c = load_model_case(base)
    cfg = c["cfg"]
    ds = c["meta"]["dataset"]
    task = {"PPI": "ppi", "PATTERN": "pattern"}.get(ds, "planetoid")
    heads = [1] + cfg["num_heads_per_layer"]
    widths = cfg["head_output_features_per_layer"]
    concat = cfg["heads_concat_per_layer"]
    add_skip = cfg["add_skip_connection"]
    L = cfg["num_layers"]
    N, C = c["x"].shape[0], cfg["num_classes"]
    y, rows = step_labels(task, N, C)
    store = {"meta": np.array(json.dumps(dict(kind="step", base=base, task=task,
                                              variants=list(variants))))}
    for vi, coef in enumerate(variants):
        mods = [ref_layer(heads[i] * widths[i], widths[i + 1], heads[i + 1], concat[i], W, a)
                for i, (W, a) in enumerate(c["layers"])]
        skips = [None if s is None else torch.from_numpy(s).requires_grad_(True)
                 for s in c["skips"]]
        xt = torch.from_numpy(c["x"])
        edge_index = torch.from_numpy(c["edge_index"])
        atts, sk = [], 0
        for i in range(L):
            layer_input = xt
            xt, (edge_index, att) = mods[i](xt, edge_index, return_attention_weights=True)
            atts.append(att)
            if add_skip[i]:
                Ws = skips[sk]
                sk += 1
                so = layer_input if Ws is None else layer_input @ Ws.T
                if concat[i]:
                    xt = xt + so
                else:
                    xt = xt + so.view(-1, heads[i + 1], widths[i + 1]).mean(dim=1)
            if i != L - 1:
                xt = torch.nn.functional.elu(xt)
        if task == "planetoid":
            idx = torch.from_numpy(rows)
            loss = torch.nn.CrossEntropyLoss(reduction="mean")(
                xt[idx], torch.from_numpy(y)[idx]) + coef * ref_attention_norm_graph(edge_index,
                                                                                     atts)
        elif task == "ppi":
            loss = torch.nn.BCEWithLogitsLoss(reduction="mean")(xt, torch.from_numpy(y))
            if coef != 0.0:
                loss = loss + coef * ref_attention_norm_graph(edge_index, atts)
        else:
            loss = torch.nn.BCEWithLogitsLoss(reduction="mean", pos_weight=torch.tensor(
                [1 / 0.1765]))(torch.squeeze(xt), torch.from_numpy(y))
        loss.backward()
        store[f"v{vi}_loss"] = np.array(loss.item(), dtype=np.float64)
        for i, m in enumerate(mods):
            put(store, f"v{vi}_grad_W{i}", m.W.weight.grad.numpy())
            put(store, f"v{vi}_grad_a{i}", m.a.weight.grad.numpy())
        for j, s in enumerate(skips):
            if s is not None:
                put(store, f"v{vi}_grad_skip{j}", s.grad.numpy())
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **store)
    print(f"{name}: task={task} N={N} variants={variants}")


def step_cases():
    for ds in ("cora", "citeseer", "pubmed"):
        step_case(f"{ds}_step_trained", f"{ds}_model_trained", [0.0, -0.5])
    step_case("ppi_step_small", "ppi_model_small", [0.0, 0.5])
    step_case("pattern_step_trained", "pattern_model_trained", [0.0])


if __name__ == "__main__" and "--steps" in sys.argv:
    torch.set_num_threads(8)
    step_cases()
elif __name__ == "__main__" and "--planetoid" in sys.argv:
    torch.set_num_threads(8)
    planetoid_model_cases()
elif __name__ == "__main__":
    if "--ppi-full-only" in sys.argv:
        torch.set_num_threads(8)
        ppi_full_cases()
    elif "--extra-only" in sys.argv:
        torch.set_num_threads(8)
        extra_cases()
    else:
        main(models_only="--models-only" in sys.argv)
