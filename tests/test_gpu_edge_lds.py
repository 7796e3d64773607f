"""The LDS-staged edge forward (csrc/edge_lds.hip, gatx.tuning edge_lds=1): concat layers on
graphs that cut into node blocks of <= 2304 nodes stage one 16-float chunk of every row of a
block in LDS and aggregate from there (records pass: den, alpha, max() ties and per-edge
{row, alpha~} records). Parity: every reference golden (layers, models, task steps' gradients
through the unchanged backward) as test_gpu_layer.py checks them, and the L2-gather pass's results
to fp32 summation order on the headline batch."""
import numpy as np
import pytest
import torch

from golden_io import LAYER_CASES, MODEL_CASES

pytestmark = pytest.mark.gpu


@pytest.fixture
def lds_on():
    from gatx import tuning
    tuning.set(edge_lds=1, lds_min_edges=0)   # every size: the goldens are small graphs
    yield
    tuning.reset()


def _took_lds(c, device):
    """Whether this golden's layer takes the LDS-staged pass (concat, <= 8 heads, blocks fit)."""
    import gatx
    from gatx import functional as gf
    from gatx.graph import graph_cache
    m = c["meta"]
    ei = torch.from_numpy(np.ascontiguousarray(c["edge_index"])).to(device)
    gatx.clear_graph_cache()
    g = graph_cache.get(ei, c["x"].shape[0], m["add_self_loops"])
    sh = gf.LayerShape(m["num_heads"], m["out_features"], m["in_features"], m["concat"],
                       m["const_attention"])
    return gf.lds_blocks(g, sh) is not None and not gf.use_reassociation(sh)


@pytest.mark.parametrize("name", LAYER_CASES)
def test_layer_goldens_lds(name, device, lds_on):
    from test_gpu_layer import test_layer_matches_reference_goldens
    test_layer_matches_reference_goldens(name, device)


def test_lds_path_is_taken(device, lds_on):
    from golden_io import load_layer_case
    took = {n: _took_lds(load_layer_case(n), device) for n in
            ("ppi_small_l1", "ppi_full_l1", "edge_dropout", "edge_bias", "edge_odd_widths",
             "edge_trailing_isolated", "cora_l0_trained", "ppi_small_l2")}
    assert took["ppi_small_l1"] and took["ppi_full_l1"]
    assert not took["cora_l0_trained"]    # one 2708-node component: no block fits the image
    assert took["ppi_small_l2"]           # head mean (round 6: gatx_edge_lds_mean_forward)
    assert not took["edge_dropout"]       # narrow input: the reassociated first-layer pass


@pytest.mark.parametrize("G,n,e,fin,NH,F,dropout,concat", [
    (3, 300, 4000, 64, 2, 16, 0.0, True),       # several blocks
    (3, 300, 4000, 64, 2, 16, 0.6, True),       # attention dropout through the records
    (2, 200, 3000, 16, 3, 7, 0.0, True),        # F % 4 != 0: scalar epilogue, padded chunk
    (1, 2245, 61318, 512, 8, 64, 0.0, True),    # one full PPI-size graph, 8 heads
    (1, 2300, 20000, 64, 4, 20, 0.0, True),     # a block near the 2304-row image
    (2, 2000, 9000, 96, 4, 40, 0.3, True),      # blocks packed over two graphs
    # head mean (round 6, gatx_edge_lds_mean_forward): heads staged in turn, the mean in registers
    (3, 300, 4000, 64, 6, 16, 0.0, False),      # several blocks, one range each
    (1, 2245, 61318, 256, 6, 121, 0.0, False),  # PPI L2's shape on one full graph: 3 ranges,
                                                # a partial last chunk (124 = 7.75 x 16)
    (2, 2000, 9000, 96, 4, 40, 0.3, False),     # attention dropout, blocks over two graphs
    (1, 2300, 20000, 64, 3, 20, 0.0, False),    # a block near the 2304-row image
    (3, 300, 3000, 16, 1, 1, 0.0, False),       # PATTERN's last layer: one head, one feature
    (2, 200, 3000, 16, 8, 7, 0.0, False),       # 8 heads, F % 4 != 0
])
def test_lds_vs_oracle(G, n, e, fin, NH, F, dropout, concat, device, lds_on):
    from test_gpu_layer import _layer_vs_oracle
    _layer_vs_oracle(device, G, n, e, fin, NH, F, concat, dropout=dropout)


def test_lds_mean_path_is_taken(device, lds_on):
    """The head-mean cases above really run the LDS-staged mean kernel: the host selects it for
    a head-mean layer whose graph cuts into blocks, not for one with a fused output dropout."""
    import gatx
    from gatx import data as gd
    from gatx import functional as gf
    from gatx.graph import graph_cache
    b = gd.uniform_graph_batch(1, 2245, 61318, 256, feature_seed=5)
    gatx.clear_graph_cache()
    g = graph_cache.get(torch.from_numpy(b.edge_index).to(device), b.num_nodes, True)
    sh = gf.LayerShape(6, 121, 256, False, False)
    assert gf.lds_blocks(g, sh) is not None
    assert gf.lds_blocks(g, sh, out_p=0.5) is None
    gatx.tuning.set(edge_lds_mean=0)
    assert gf.lds_blocks(g, sh) is None


@pytest.mark.parametrize("name", MODEL_CASES)
def test_model_goldens_lds(name, device, lds_on):
    from test_gpu_layer import test_model_matches_reference_goldens
    test_model_matches_reference_goldens(name, device)


def test_headline_batch_lds_equals_gather(device):
    """The 20-graph PPI batch: the LDS-staged forward against the L2-gather forward (both checked
    against the reference elsewhere) — outputs to fp32 summation order, alphas bitwise where the
    layer inputs agree (the records pass sums the denominators exactly as the gather pass does)."""
    import gatx
    from gatx import data as gd
    from gatx import tuning
    from gatx.config import data_config
    torch.manual_seed(0)
    model = gatx.GATModel(**data_config["PPI"]).to(device).eval()
    b = gd.dataset_batch("PPI", 20, graph_seed=42, feature_seed=1)
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    res = []
    for lds in (0, 1):
        tuning.set(edge_lds=lds)
        gatx.clear_graph_cache()
        with torch.no_grad():
            out, _, al = model.forward_and_return_attention(x, ei)
        res.append((out.clone(), [a.clone() for a in al]))
    tuning.reset()
    (o0, a0), (o1, a1) = res
    assert float((o0 - o1).abs().max()) <= 1e-5 * max(1.0, float(o0.abs().max()))
    # layers 0 (reassociated: the gather pass in both runs) and 1 (LDS-staged) see identical
    # inputs: their alphas agree bitwise; layer 2's input differs in the last bits
    assert torch.equal(a0[0], a1[0]) and torch.equal(a0[1], a1[1])
    assert float((a0[2] - a1[2]).abs().max()) <= 1e-6


def test_captured_forward_lds(device, lds_on):
    """A captured forward that rebuilds its CSR every replay takes the LDS path once the
    edge_index's blocks are known (decided by the warm-up), and replays equal the eager step."""
    import gatx
    from gatx import data as gd
    from gatx.capture import CapturedStep
    from gatx.config import data_config
    torch.manual_seed(0)
    model = gatx.GATModel(**data_config["PPI"]).to(device).eval()
    b = gd.dataset_batch("PPI", 3, graph_seed=5, feature_seed=6)
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)

    def step():
        gatx.clear_graph_cache()
        with torch.no_grad():
            return model(x, ei)

    ref = step().clone()
    cap = CapturedStep(step)
    for _ in range(5):
        out = cap()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_captured_forward_lds_interleaved(device, lds_on):
    """Replays that each follow a kernel launched outside the graph (a torch fill, as bench.py's
    fallback-counter read and region marks): the node blocks are recomputed in every replay and
    the LDS pass must see them (round 5: a memset + atomic counter read by the next kernel came
    back stale on exactly these replays, so the pass skipped its work)."""
    import gatx
    from gatx import data as gd
    from gatx.capture import CapturedStep
    from gatx.config import data_config
    from gatx.graph import graph_cache
    torch.manual_seed(0)
    model = gatx.GATModel(**data_config["PPI"]).to(device).eval()
    b = gd.dataset_batch("PPI", 3, graph_seed=5, feature_seed=6)
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)

    def step():
        gatx.clear_graph_cache()
        with torch.no_grad():
            return model(x, ei)

    ref = step().clone()
    cap = CapturedStep(step)
    segs, count = graph_cache.get(ei, b.num_nodes, True)._hub_plans[("blocks", 2304)]
    for _ in range(4):
        torch.zeros(1, device=device)
        out = cap()
        torch.cuda.synchronize()
        assert int(count.item()) == 3   # the round-5 failure left -1 here
        assert torch.equal(out, ref)


def _blocked_edges(N, E, runs, seed):
    """E random edges that stay inside consecutive node runs of the given lengths."""
    rng = np.random.default_rng(seed)
    starts = np.concatenate([[0], np.cumsum(runs)[:-1]])
    which = rng.integers(0, len(runs), E)
    lo = starts[which]
    ln = np.asarray(runs)[which]
    src = lo + rng.integers(0, ln)
    dst = lo + rng.integers(0, ln)
    assert starts[-1] + runs[-1] == N
    return np.stack([src, dst]).astype(np.int64)


def test_captured_forward_lds_blocks_change(device, lds_on):
    """A captured LDS forward replayed on edges copied into its edge_index whose node blocks no
    longer match the launch (more blocks than the grid holds, then none at all): the pass falls
    back to gathering rows from global memory and still equals the eager (L2-gather) step."""
    import gatx
    from gatx import tuning
    from gatx.capture import CapturedStep
    from gatx.config import data_config
    torch.manual_seed(0)
    model = gatx.GATModel(**data_config["PPI"]).to(device).eval()
    N, E = 4490, 60000
    x = torch.randn(N, 50, device=device)
    ei = torch.from_numpy(_blocked_edges(N, E, [2245, 2245], 1)).to(device)

    def step():
        gatx.clear_graph_cache()
        with torch.no_grad():
            return model(x, ei)

    cap = CapturedStep(step)
    out = cap().clone()
    tuning.set(edge_lds=0)
    assert float((out - step()).abs().max()) <= 1e-5
    tuning.set(edge_lds=1)
    for runs in ([1200, 1200, 1200, 890], [N]):   # 4 blocks > the grid's 2; one 4490-node run
        ei.copy_(torch.from_numpy(_blocked_edges(N, E, runs, 2)).to(device))
        out = cap().clone()
        tuning.set(edge_lds=0)
        ref = step()
        tuning.set(edge_lds=1)
        assert float((out - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("side", [0, 1])
def test_side_stream_model_equals_serial(side, device):
    """tuning side_stream (node blocks and GATModel's non-final alpha passes on a second stream,
    joined before use): the PPI model's outputs and every alpha equal the one-stream run bitwise,
    eager and captured, forward and a training step's gradients."""
    import gatx
    from gatx import data as gd
    from gatx import tuning
    from gatx.capture import CapturedStep
    from gatx.config import data_config
    b = gd.dataset_batch("PPI", 3, graph_seed=9, feature_seed=10)
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    res = []
    for sd in (0, side):
        tuning.set(side_stream=sd, lds_min_edges=0)
        torch.manual_seed(0)
        model = gatx.GATModel(**data_config["PPI"]).to(device)
        gatx.clear_graph_cache()
        with torch.no_grad():
            out, _, al = model.eval().forward_and_return_attention(x, ei)

        def step():
            gatx.clear_graph_cache()
            with torch.no_grad():
                return model(x, ei)
        cap = CapturedStep(step)
        rep = cap().clone()
        model.train()
        gatx.clear_graph_cache()
        o, ei2, al2 = model.forward_and_return_attention(x, ei)
        (o.square().mean() + 0.1 * model.calc_attention_norm(ei2, al2)).backward()
        res.append((out.clone(), [a.clone() for a in al], rep,
                    [p.grad.clone() for p in model.parameters()]))
    tuning.reset()
    (o0, a0, r0, g0), (o1, a1, r1, g1) = res
    assert torch.equal(o0, o1) and torch.equal(r0, r1) and torch.equal(r0, o0)
    assert all(torch.equal(u, v) for u, v in zip(a0, a1))
    assert all(torch.equal(u, v) for u, v in zip(g0, g1))


def test_lds_output_dropout_training_equals_gather(device, lds_on):
    """GATModel training with input dropout: the next layer's dropout rides on the LDS pass's
    epilogue (edge_lds_kernel<.., DROP=true>, gatx's counter-based mask): outputs, alphas and every
    parameter gradient equal the L2-gather pass's to fp32 summation order."""
    import gatx
    from gatx import data as gd
    from gatx import tuning
    from gatx.config import data_config
    cfg = dict(data_config["PPI"])
    cfg["dropout"] = 0.3
    b = gd.dataset_batch("PPI", 3, graph_seed=13, feature_seed=14)
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    res = []
    for lds in (1, 0):
        tuning.set(edge_lds=lds)
        torch.manual_seed(0)
        model = gatx.GATModel(**cfg).to(device).train()
        gatx.clear_graph_cache()
        torch.manual_seed(1)              # the per-layer dropout seeds
        out, ei2, al = model.forward_and_return_attention(x, ei)
        (out.square().mean() + 0.1 * model.calc_attention_norm(ei2, al)).backward()
        res.append((out.detach().clone(), [a.detach().clone() for a in al],
                    [p.grad.clone() for p in model.parameters()]))
    (o1, a1, g1), (o0, a0, g0) = res
    scale = max(1.0, float(o0.abs().max()))
    assert float((o1 - o0).abs().max()) <= 1e-5 * scale
    assert all(float((u - v).abs().max()) <= 1e-6 for u, v in zip(a1, a0))
    for u, v in zip(g1, g0):
        assert float((u - v).abs().max()) <= 1e-4 * max(1.0, float(v.abs().max()))


def test_side_alpha_pass_keeps_its_buffers(device, monkeypatch):
    """The side-stream alpha pass of a no_grad forward (tuning side_stream=1) reads S, M_ord, den
    and writes argmax / alpha after the caller has dropped them: a delayed pass (a sleep on the
    side stream ahead of it) must still read its own buffers, not blocks the caching allocator
    handed to the next layer's projection GEMM (functional._alpha_pass records them on the side
    stream). Alphas and outputs equal the one-stream forward bitwise."""
    import gatx
    from gatx import data as gd
    from gatx import functional as gf
    from gatx import tuning
    from gatx.config import data_config
    b = gd.dataset_batch("PPI", 3, graph_seed=19, feature_seed=20)
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    torch.manual_seed(0)
    model = gatx.GATModel(**data_config["PPI"]).to(device).eval()
    res = []
    orig = gf._attention_alpha

    def delayed(*a, **k):
        torch.cuda._sleep(20_000_000)   # ~10 ms on the stream the pass runs on
        return orig(*a, **k)

    try:
        for sd in (0, 1):
            tuning.set(side_stream=sd, lds_min_edges=0)
            if sd:
                monkeypatch.setattr(gf, "_attention_alpha", delayed)
            gatx.clear_graph_cache()
            with torch.no_grad():
                out, _, al = model.forward_and_return_attention(x, ei)
            torch.cuda.synchronize()
            res.append((out.clone(), [a.clone() for a in al]))
    finally:
        tuning.reset()
    (o0, a0), (o1, a1) = res
    assert torch.equal(o0, o1)
    for u, v in zip(a0, a1):
        assert torch.equal(u, v)


@pytest.mark.parametrize("dropout", [0.0, 0.3])
def test_lds_backward_source_pass_equals_gather(dropout, device, lds_on):
    """tuning edge_lds_bwd (round 6): the backward's source pass of the concat layers as the LDS
    walk over go's rows with transposed records (gatx_edge_records_src) equals the L2-gather
    source pass — every parameter gradient and the input gradient, to fp32 summation order (the
    walk adds each destination's terms in another fixed order); g_s_src is bitwise the same. With
    dropout the records carry the attention dropout mask."""
    import gatx
    from gatx import data as gd
    from gatx import tuning
    torch.manual_seed(0)
    model = gatx.GATModel(num_classes=16, num_input_node_features=48, num_layers=3,
                          num_heads_per_layer=[4, 4, 6], heads_concat_per_layer=[True, True, False],
                          head_output_features_per_layer=[48, 64, 64, 16],
                          add_skip_connection=[False, True, False], dropout=dropout).to(device)
    model.train()
    b = gd.uniform_graph_batch(3, 1500, 30000, 48, feature_seed=2)
    x0 = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    g_out = torch.randn(b.num_nodes, 16, device=device, generator=torch.Generator(device=device).manual_seed(5))
    grads = []
    for on in (0, 1):
        tuning.set(edge_lds_bwd=on)
        gatx.clear_graph_cache()
        model.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        torch.manual_seed(7)   # the same dropout seeds in both runs
        out = model(x, ei)
        out.backward(g_out)
        grads.append([x.grad.clone()] + [p.grad.clone() for p in model.parameters()])
    for a, c in zip(*grads):
        scale = max(1.0, c.abs().max().item())
        assert (a - c).abs().max().item() <= 2e-5 * scale
