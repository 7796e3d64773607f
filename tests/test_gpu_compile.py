"""torch.compile over gatx models through the registered ops (gatx/ops.py): fullgraph=True (no
graph breaks), results equal to the eager gatx path — which the golden tests pin to the
reference — bit for bit (the same kernels run in the same order)."""
import pytest
import torch

from gatx import data as gd

pytestmark = pytest.mark.gpu


def _ppi_model(device, layers=3):
    from gatx import GATModel
    from gatx.config import data_config
    cfg = dict(data_config["PPI"])
    if layers == 2:   # the first two PPI layers: 50 -> 4x256 concat -> 6x121 mean
        cfg.update(num_layers=2, num_heads_per_layer=[4, 6], heads_concat_per_layer=[True, False],
                   head_output_features_per_layer=[50, 256, 121], add_skip_connection=[False, True])
    torch.manual_seed(0)
    return GATModel(**cfg).to(device), cfg


def _batch(device, cfg, G=2, n=256, e=4000):
    b = gd.uniform_graph_batch(G, n, e, cfg["num_input_node_features"], feature_seed=3)
    return torch.from_numpy(b.x).to(device), torch.from_numpy(b.edge_index).to(device)


@pytest.mark.parametrize("layers", [2, 3])
def test_compiled_forward_equals_eager(layers, device):
    from gatx import clear_graph_cache
    model, cfg = _ppi_model(device, layers)
    model.eval()
    x, ei = _batch(device, cfg)
    with torch.no_grad():
        ref = model(x, ei)
        clear_graph_cache()
        fn = torch.compile(model, fullgraph=True, backend="inductor")
        out = fn(x, ei)
        out2 = fn(x, ei)   # second call: cached graph, warm caches
    torch.cuda.synchronize()
    if layers == 3:   # only gatx ops in the graph (PPI's skip is the identity): bit for bit
        assert torch.equal(out, ref) and torch.equal(out2, ref)
    else:   # the Linear skip + head mean run as inductor code (its own mm / reduction order)
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(out2, ref, rtol=1e-5, atol=1e-5)


def test_compiled_train_step_equals_eager(device):
    """PPI_GAT.training_step shape (models/ppi_gat.py:15-33): forward_and_return_attention, BCE,
    the attention norm, backward — compiled with AOTAutograd (fwd + bwd graphs, no codegen: the
    same aten kernels as eager around the gatx ops) == eager."""
    from gatx import clear_graph_cache
    model, cfg = _ppi_model(device, 3)   # identity skip: every op is the same kernel in both
    model.train()
    x, ei = _batch(device, cfg)
    y = (torch.rand(x.size(0), 121, device=device, generator=torch.Generator(device=device)
                    .manual_seed(1)) > 0.5).float()

    def step(m, xx):
        out, ei2, atts = m.forward_and_return_attention(xx, ei)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(out, y)
        return loss + 0.1 * m.calc_attention_norm(ei2, atts)

    def grads(fn):
        model.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        loss = fn(model, xx)
        loss.backward()
        return loss.detach(), xx.grad, [p.grad.clone() for p in model.parameters()]

    l0, gx0, gp0 = grads(step)
    clear_graph_cache()
    l1, gx1, gp1 = grads(torch.compile(step, fullgraph=True, backend="aot_eager"))
    torch.cuda.synchronize()
    assert torch.equal(l0, l1)
    assert torch.equal(gx0, gx1)
    for a, b in zip(gp0, gp1):
        assert torch.equal(a, b)


def test_op_direct_call_matches_layer(device):
    """torch.ops.gatx.layer_fwd called directly == GATLayer.forward (return contract)."""
    from gatx import GATLayer
    torch.manual_seed(0)
    layer = GATLayer(32, 16, 4, True, add_self_loops=True).to(device)
    b = gd.uniform_graph_batch(1, 200, 3000, 32, feature_seed=3)
    x, ei = torch.from_numpy(b.x).to(device), torch.from_numpy(b.edge_index).to(device)
    out, (ei2, alpha) = layer(x, ei, return_attention_weights=True)
    o2, e2, a2, state = torch.ops.gatx.layer_fwd(x, ei, layer.W.weight, layer.a.weight, None, None,
                                                 None, 4, 16, True, True, False, 0.0, False)
    assert torch.equal(out, o2) and torch.equal(ei2, e2) and torch.equal(alpha, a2)
    assert len(state) == 8
