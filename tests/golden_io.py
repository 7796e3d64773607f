"""Load the golden fixtures written by tests/golden/make_goldens.py (data only: inputs regenerate
from splitmix64 seeds via gatx.data when they were too big to store)."""
from __future__ import annotations

import glob
import json
import os

import numpy as np

from gatx import data as gdata

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LAYER_CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                     if "_model_" not in os.path.basename(p)
                     and "_step_" not in os.path.basename(p))
MODEL_CASES = ["pattern_model_trained", "ppi_model_small", "cora_model_trained",
               "citeseer_model_trained", "pubmed_model_trained"]


def _gen_batch(gen):
    b = gdata.uniform_graph_batch(gen["G"], gen["n"], gen["e"], gen["in_features"],
                                  graph_seed=gen.get("graph_seed", 42),
                                  feature_seed=gen.get("feature_seed", 1),
                                  features=gen.get("features", "normal"))
    return b.x, b.edge_index


class Expected:
    """An expected array: full, or a row sample + checksums (sum, sum|.|, sum^2, max|.|)."""

    def __init__(self, z, name):
        self.name = name
        if name in z:
            self.full, self.rows, self.sample, self.checksums = z[name], None, None, None
        else:
            self.full = None
            self.rows = z[f"{name}__rows"]
            self.sample = z[f"{name}__sample"]
            self.checksums = z[f"{name}__checksums"]

    def scale(self):
        return float(np.abs(self.full).max()) if self.full is not None else float(self.checksums[3])

    def check(self, got, atol, rtol_scale=False, what=""):
        """max|got - ref| <= atol * (max(1, max|ref|) if rtol_scale else 1)."""
        got = np.asarray(got, dtype=np.float64)
        tol = atol * (max(1.0, self.scale()) if rtol_scale else 1.0)
        if self.full is not None:
            assert got.shape == self.full.shape, (what, self.name, got.shape, self.full.shape)
            err = float(np.abs(got - self.full).max()) if got.size else 0.0
            assert err <= tol, f"{what}{self.name}: max|d|={err:.3e} > {tol:.3e}"
            return err
        err = float(np.abs(got[self.rows] - self.sample).max())
        assert err <= tol, f"{what}{self.name}[rows]: max|d|={err:.3e} > {tol:.3e}"
        cs = np.array([got.sum(), np.abs(got).sum(), (got * got).sum(), np.abs(got).max()])
        # checksums: relative agreement, with slack for the accumulated fp32 noise of a big array
        n = got.size
        assert abs(cs[0] - self.checksums[0]) <= tol * np.sqrt(n) * 4 + 1e-6 * abs(self.checksums[1]), \
            f"{what}{self.name}: sum {cs[0]} vs {self.checksums[0]}"
        for i in (1, 2, 3):
            r = abs(cs[i] - self.checksums[i]) / max(abs(self.checksums[i]), 1e-30)
            assert r <= 1e-4, f"{what}{self.name}: checksum[{i}] rel {r:.2e}"
        return err


def load_layer_case(name):
    z = np.load(os.path.join(GOLDEN_DIR, f"{name}.npz"))
    meta = json.loads(str(z["meta"]))
    if "x" in z:
        x, ei = z["x"], z["edge_index"]
    else:
        x, ei = _gen_batch(meta["gen"])
    if meta["edge_dtype"] == "int32":
        ei = ei.astype(np.int32)
    NH, F, fin = meta["num_heads"], meta["out_features"], meta["in_features"]
    if meta.get("wgen"):
        sw, sa = meta["wgen"]
        W = gdata.xavier_uniform(sw, NH * F, fin)
        a = gdata.xavier_uniform(sa, NH, NH * 2 * F)
    else:
        W = z["W"]
        a = z["a"] if "a" in z else None
    bias = z["bias"] if "bias" in z else None
    exp = {k: Expected(z, k) for k in ("out", "alpha", "grad_x", "grad_W", "grad_a", "grad_bias")
           if k in z or f"{k}__rows" in z}
    return dict(meta=meta, x=x, edge_index=ei, W=W, a=a, bias=bias, expected=exp,
                edge_index_out=z["edge_index_out"])


def grad_seeds(out_shape, alpha_shape):
    """The upstream gradients make_goldens.py used."""
    g_out = gdata.normal(7, int(np.prod(out_shape))).reshape(out_shape)
    g_alpha = 0.1 * gdata.normal(8, int(np.prod(alpha_shape))).reshape(alpha_shape)
    return g_out, g_alpha


def load_model_case(name):
    z = np.load(os.path.join(GOLDEN_DIR, f"{name}.npz"))
    meta = json.loads(str(z["meta"]))
    x, ei = _gen_batch(meta["gen"])
    from gatx.config import data_config
    cfg = data_config[meta["dataset"]]
    heads = [1] + cfg["num_heads_per_layer"]
    widths = cfg["head_output_features_per_layer"]
    L = cfg["num_layers"]
    layers = []
    for i in range(L):
        if meta.get("wgen"):
            sw, sa = meta["wgen"][i]
            fin, F, NH = heads[i] * widths[i], widths[i + 1], heads[i + 1]
            layers.append((gdata.xavier_uniform(sw, NH * F, fin),
                           gdata.xavier_uniform(sa, NH, NH * 2 * F)))
        else:
            layers.append((z[f"W{i}"], z[f"a{i}"]))
    skips = []
    for i, s in enumerate(cfg["add_skip_connection"]):
        if s:
            skips.append(z[f"skip{len(skips)}"] if f"skip{len(skips)}" in z else None)
    exp = {"out": Expected(z, "out")}
    for i in range(L):
        exp[f"alpha{i}"] = Expected(z, f"alpha{i}")
        if f"attention_norm_grad{i}" in z or f"attention_norm_grad{i}__rows" in z:
            exp[f"attention_norm_grad{i}"] = Expected(z, f"attention_norm_grad{i}")
    if "attention_norm" in z:
        exp["attention_norm"] = float(z["attention_norm"])
    return dict(meta=meta, cfg=cfg, x=x, edge_index=ei, layers=layers, skips=skips,
                expected=exp, edge_index_out=z["edge_index_out"])


STEP_CASES = ["cora_step_trained", "citeseer_step_trained", "pubmed_step_trained",
              "ppi_step_small", "pattern_step_trained"]


def step_labels(task, N, C):
    """The synthetic labels make_goldens.step_labels drew (targets, labelled rows or None)."""
    if task == "planetoid":
        return (gdata.randint(123, N, 1 << 30) % C).astype(np.int64), np.arange(20 * C)
    if task == "ppi":
        return gdata.randint(124, N * C, 2).reshape(N, C).astype(np.float32), None
    return gdata.randint(125, N, 2).astype(np.float32), None


def load_step_case(name):
    """A training-step golden (make_goldens.step_case): the base model case's inputs and weights,
    the task's labels, and per variant (reward / penalty) the reference's loss and gradients."""
    z = np.load(os.path.join(GOLDEN_DIR, f"{name}.npz"))
    meta = json.loads(str(z["meta"]))
    c = load_model_case(meta["base"])
    cfg = c["cfg"]
    N = c["x"].shape[0]
    labels, rows = step_labels(meta["task"], N, cfg["num_classes"])
    variants = []
    for vi, coef in enumerate(meta["variants"]):
        exp = {"loss": float(z[f"v{vi}_loss"])}
        for i in range(cfg["num_layers"]):
            exp[f"W{i}"] = Expected(z, f"v{vi}_grad_W{i}")
            exp[f"a{i}"] = Expected(z, f"v{vi}_grad_a{i}")
        for j in range(len(c["skips"])):
            if f"v{vi}_grad_skip{j}" in z or f"v{vi}_grad_skip{j}__rows" in z:
                exp[f"skip{j}"] = Expected(z, f"v{vi}_grad_skip{j}")
        variants.append((coef, exp))
    return dict(c, task=meta["task"], labels=labels, rows=rows, variants=variants)
