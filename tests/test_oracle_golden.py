"""Pin the CPU oracle (oracle/gat_oracle.py) to the reference's own outputs (tests/golden/*.npz,
produced by importing /root/reference/models/gat_layer.py — see tests/golden/make_goldens.py)."""
import numpy as np
import pytest

from golden_io import (LAYER_CASES, MODEL_CASES, STEP_CASES, grad_seeds, load_layer_case,
                       load_model_case, load_step_case)
from oracle import gat_oracle as orc

OUT_TOL = 1e-4          # outputs / alpha: absolute (north_star: within 1e-4 fp32)
GRAD_TOL = 1e-4         # grads: max|d| <= 1e-4 * max(1, max|ref|)  


def run_oracle(c, dtype=np.float32):
    m = c["meta"]
    keep = None
    if m["dropout"] > 0:
        E2 = c["edge_index_out"].shape[1]
        keep = orc.dropout_keep(m["seed"], E2, m["num_heads"], m["dropout"])
    out, ei2, alpha, cache = orc.gat_layer_forward(
        c["x"], c["edge_index"], c["W"], c["a"], m["num_heads"], m["out_features"], m["concat"],
        bias=c["bias"], add_self_loops=m["add_self_loops"], const_attention=m["const_attention"],
        dropout_p=m["dropout"], keep=keep, dtype=dtype)
    g_out, g_alpha = grad_seeds(out.shape, alpha.shape)
    grads = orc.gat_layer_backward(cache, g_out, g_alpha if m["use_g_alpha"] else None)
    return out, ei2, alpha, grads


@pytest.mark.parametrize("name", LAYER_CASES)
def test_oracle_matches_reference_layer(name):
    c = load_layer_case(name)
    out, ei2, alpha, grads = run_oracle(c)
    e = c["expected"]
    np.testing.assert_array_equal(ei2, c["edge_index_out"])
    e["out"].check(out, OUT_TOL)
    e["alpha"].check(alpha, OUT_TOL)
    e["grad_x"].check(grads["x"], GRAD_TOL, rtol_scale=True)
    e["grad_W"].check(grads["W"], GRAD_TOL, rtol_scale=True)
    if "grad_a" in e:
        e["grad_a"].check(grads["a"], GRAD_TOL, rtol_scale=True)
    if "grad_bias" in e:
        e["grad_bias"].check(grads["bias"], GRAD_TOL, rtol_scale=True)


@pytest.mark.parametrize("name", ["adversarial_a1e3", "edge_ties_a_zero", "edge_dropout"])
def test_oracle_fp64_agrees(name):
    """The fp64 oracle agrees with the fp32 reference too (guards against matching fp32 noise)."""
    c = load_layer_case(name)
    out, _, alpha, grads = run_oracle(c, dtype=np.float64)
    c["expected"]["out"].check(out, OUT_TOL)
    c["expected"]["grad_W"].check(grads["W"], GRAD_TOL, rtol_scale=True)


@pytest.mark.parametrize("name", MODEL_CASES)
def test_oracle_matches_reference_model(name):
    c = load_model_case(name)
    cfg = c["cfg"]
    out, ei2, alphas = orc.gat_model_forward(
        c["x"], c["edge_index"], c["layers"], c["skips"], cfg["num_heads_per_layer"],
        cfg["head_output_features_per_layer"][1:], cfg["heads_concat_per_layer"],
        cfg["add_skip_connection"])
    np.testing.assert_array_equal(ei2, c["edge_index_out"])
    c["expected"]["out"].check(out, OUT_TOL)
    for i, al in enumerate(alphas):
        c["expected"][f"alpha{i}"].check(al, OUT_TOL)


@pytest.mark.parametrize("name", MODEL_CASES)
def test_oracle_attention_norm_matches_reference(name):
    """calc_attention_norm (models/GATModel.py:189-230) and its gradient on the reference's own
    alphas / edge_index' (goldens made with the reference's sum_over_neighbourhood)."""
    c = load_model_case(name)
    e = c["expected"]
    L = len(c["layers"])
    alphas = [e[f"alpha{i}"].full for i in range(L)]
    own = any(a is None for a in alphas)
    if own:
        # a golden alpha too big to store in full (Pubmed): the oracle's own alphas, which
        # test_oracle_matches_reference_model pins to the golden's rows and checksums
        cfg = c["cfg"]
        _, _, alphas = orc.gat_model_forward(
            c["x"], c["edge_index"], c["layers"], c["skips"], cfg["num_heads_per_layer"],
            cfg["head_output_features_per_layer"][1:], cfg["heads_concat_per_layer"],
            cfg["add_skip_connection"])
    ei = c["edge_index_out"]
    v = orc.calc_attention_norm(ei, alphas)
    # fp32 summation-order noise of torch.norm over ~5e4 terms: relative 1e-5
    assert abs(v - e["attention_norm"]) <= 1e-5 * max(1.0, abs(e["attention_norm"]))
    if own:
        # sgn(alpha * deg - 1) flips wherever the two fp32 alphas straddle the kink: the
        # gradient is only comparable on the reference's own alphas
        return
    for i, g in enumerate(orc.calc_attention_norm_grad(ei, alphas)):
        e[f"attention_norm_grad{i}"].check(g, 1e-9)


def test_self_loop_rewrite_order():
    ei = np.array([[0, 1, 2, 2, 4], [1, 1, 0, 2, 3]])
    got = orc.add_remaining_self_loops(ei)
    np.testing.assert_array_equal(got, [[0, 2, 4, 0, 1, 2, 3, 4], [1, 0, 3, 0, 1, 2, 3, 4]])


def test_empty_edge_index_raises():
    with pytest.raises(RuntimeError):
        orc.add_remaining_self_loops(np.zeros((2, 0), dtype=np.int64))


def test_oracle_model_backward_finite_differences():
    """gat_model_forward_backward (layer backward chained through ELU, concat / head-mean skip
    adds and skip projections) against central differences in fp64 on a tiny 3-layer model."""
    from gatx import data as gd
    rng = np.random.default_rng(3)
    N, E = 12, 40
    ei = np.stack([rng.integers(0, N, E), rng.integers(0, N, E)])
    x = rng.standard_normal((N, 5))
    heads, widths, concat = [2, 2, 3], [4, 3, 2], [True, True, False]
    add_skip = [True, True, True]
    fins = [5, 8, 6]
    layers = [(rng.standard_normal((h * f, fin)) * 0.5, rng.standard_normal((h, h * 2 * f)) * 0.5)
              for h, f, fin in zip(heads, widths, fins)]
    skips = [rng.standard_normal((8, 5)) * 0.5, rng.standard_normal((6, 8)) * 0.5, None]
    g = rng.standard_normal((N, 2))

    def loss():
        out, _, _ = orc.gat_model_forward(x, ei, layers, skips, heads, widths, concat, add_skip,
                                          dtype=np.float64)
        return float((out * g).sum())

    _, grads = orc.gat_model_forward_backward(x, ei, layers, skips, heads, widths, concat,
                                              add_skip, g)
    eps = 1e-6
    for li in range(3):
        for which, k in ((0, "W"), (1, "a")):
            arr = layers[li][which]
            for idx in [(0, 0), (arr.shape[0] - 1, arr.shape[1] - 1), (1, 2)]:
                old = arr[idx]
                arr[idx] = old + eps
                lp = loss()
                arr[idx] = old - eps
                lm = loss()
                arr[idx] = old
                fd = (lp - lm) / (2 * eps)
                assert abs(fd - grads[k][li][idx]) <= 1e-5 * max(1.0, abs(fd)), (li, k, idx)
    for j in (0, 1):
        arr = skips[j]
        for idx in [(0, 0), (arr.shape[0] - 1, arr.shape[1] - 1)]:
            old = arr[idx]
            arr[idx] = old + eps
            lp = loss()
            arr[idx] = old - eps
            lm = loss()
            arr[idx] = old
            fd = (lp - lm) / (2 * eps)
            assert abs(fd - grads["skip"][j][idx]) <= 1e-5 * max(1.0, abs(fd)), ("skip", j, idx)


def test_oracle_planetoid_step_finite_differences():
    """planetoid_step_grads (CE over the train rows + attention_reward * calc_attention_norm,
    models/planetoid_gat.py:15-30) against central differences in fp64 on a tiny 2-layer model.
    The L1 norm is differentiated away from its kinks (no alpha * deg == 1 here)."""
    rng = np.random.default_rng(5)
    N, E = 14, 50
    ei = np.stack([rng.integers(0, N, E), rng.integers(0, N, E)])
    x = rng.standard_normal((N, 6))
    heads, widths, concat = [3, 1], [4, 5], [True, False]
    layers = [(rng.standard_normal((3 * 4, 6)) * 0.5, rng.standard_normal((3, 3 * 8)) * 0.5),
              (rng.standard_normal((5, 12)) * 0.5, rng.standard_normal((1, 10)) * 0.5)]
    labels = rng.integers(0, 5, N)
    rows = np.array([0, 3, 4, 7, 11])
    reward = -0.7

    def loss():
        v, _ = orc.planetoid_step_grads(x, ei, layers, heads, widths, concat, labels, rows, reward)
        return v

    _, grads = orc.planetoid_step_grads(x, ei, layers, heads, widths, concat, labels, rows, reward)
    eps = 1e-6
    for li in range(2):
        for which, k in ((0, "W"), (1, "a")):
            arr = layers[li][which]
            for idx in [(0, 0), (arr.shape[0] - 1, arr.shape[1] - 1), (0, 3)]:
                old = arr[idx]
                arr[idx] = old + eps
                lp = loss()
                arr[idx] = old - eps
                lm = loss()
                arr[idx] = old
                fd = (lp - lm) / (2 * eps)
                assert abs(fd - grads[k][li][idx]) <= 1e-5 * max(1.0, abs(fd)), (li, k, idx, fd)


@pytest.mark.parametrize("name", STEP_CASES)
def test_oracle_step_matches_reference(name):
    """the oracle's whole training step (model_step_grads: the task module's
    loss through the GATModel wiring and every layer's backward, in fp64) against the reference's
    own autograd (tests/golden/*_step_*.npz: reference GATLayers wired as GATModel, the task
    module's loss, `loss.backward()`), for every variant (attention reward / penalty). Model-level
    tolerance: 2e-4 of the gradient's scale (the reference's fp32 noise grows with depth)."""
    c = load_step_case(name)
    cfg = c["cfg"]
    for coef, exp in c["variants"]:
        loss, grads = orc.model_step_grads(
            c["task"], c["x"], c["edge_index"], c["layers"], c["skips"],
            cfg["num_heads_per_layer"], cfg["head_output_features_per_layer"][1:],
            cfg["heads_concat_per_layer"], cfg["add_skip_connection"], c["labels"], c["rows"],
            coef)
        assert abs(loss - exp["loss"]) <= 1e-5 * max(1.0, abs(exp["loss"])), (coef, loss)
        for i in range(cfg["num_layers"]):
            exp[f"W{i}"].check(grads["W"][i], 2e-4, rtol_scale=True, what=f"{coef} ")
            exp[f"a{i}"].check(grads["a"][i], 2e-4, rtol_scale=True, what=f"{coef} ")
        for j, g in enumerate(grads["skip"]):
            if f"skip{j}" in exp:
                exp[f"skip{j}"].check(g, 2e-4, rtol_scale=True, what=f"{coef} ")
