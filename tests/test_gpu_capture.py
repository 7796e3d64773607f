"""hipGraph capture of whole gatx steps (gatx.capture.CapturedStep): every launch of the graph
build, forward, backward and optimizer step is replayed from one graph. Replays must equal the
eager step bit for bit, many times over (a captured counter that is reset outside the graph,
like rocPRIM onesweep's block-id reset, only breaks after several replays), and the captured
graph build must rebuild from whatever edge_index holds at replay time."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(ds, G, device, seed=7):
    from gatx import data as gd
    b = gd.dataset_batch(ds, G, graph_seed=seed, feature_seed=seed + 1)
    return (torch.from_numpy(b.x).to(device), torch.from_numpy(b.edge_index).to(device), b)


@pytest.mark.parametrize("ds,G", [("PPI", 2), ("PATTERN", 8)])
def test_captured_forward_replays_equal_eager(ds, G, device):
    import gatx
    from gatx.capture import CapturedStep
    from gatx.config import data_config
    torch.manual_seed(0)
    model = gatx.GATModel(**data_config[ds]).to(device).eval()
    x, ei, _ = _batch(ds, G, device)

    def step():
        gatx.clear_graph_cache()   # the captured step rebuilds the CSR every replay
        with torch.no_grad():
            return model(x, ei)

    ref = step().clone()
    cap = CapturedStep(step)
    for _ in range(25):
        out = cap()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # new edges copied into the static edge_index: the replayed build follows them
    x2, ei2, _ = _batch(ds, G, device, seed=11)
    ei.copy_(ei2)
    x.copy_(x2)
    out = cap().clone()
    gatx.clear_graph_cache()
    with torch.no_grad():
        ref2 = model(x, ei)
    assert torch.equal(out, ref2)


def test_captured_pattern_train_step_equals_eager(device):
    """PatternGAT.training_step (models/pattern_gat.py:18-25) with Adam(capturable=True):
    parameters after k replayed steps == after k eager steps."""
    import gatx
    from gatx.capture import CapturedStep
    from gatx.config import data_config
    cfg = data_config["PATTERN"]
    x, ei, b = _batch("PATTERN", 8, device)
    y = (torch.from_numpy(np.arange(b.num_nodes) % 6 == 0).float()).to(device)
    loss_fn = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([1 / 0.1765], device=device))

    def make():
        torch.manual_seed(0)
        m = gatx.GATModel(**cfg).to(device).train()
        o = torch.optim.Adam(m.parameters(), lr=cfg["learning_rate"], capturable=True)
        return m, o

    def make_step(m, o):
        def step():
            gatx.clear_graph_cache()
            o.zero_grad(set_to_none=True)
            out = m(x, ei).squeeze(-1)
            loss = loss_fn(out, y)
            loss.backward()
            o.step()
            return loss.detach()
        return step

    m1, o1 = make()
    s1 = make_step(m1, o1)
    losses = [float(s1()) for _ in range(2 + 6)]   # CapturedStep warms up twice, then 6 replays
    m2, o2 = make()
    import warnings
    with warnings.catch_warnings():
        # the captured backward must accumulate on the stream that created the AccumulateGrad
        # nodes (CapturedStep: warm-ups and capture on one stream), not across streams
        warnings.filterwarnings("error", message=".*AccumulateGrad node's stream")
        cap = CapturedStep(make_step(m2, o2), warmup=2)   # capture itself runs no step
        for _ in range(6):
            last = cap()
        torch.cuda.synchronize()
    # capture ran the step once more (the captured pass's own work is not executed at capture),
    # so the 6 replays are steps 3..8, like the eager run's last six
    assert abs(float(last) - losses[-1]) <= 1e-6 * max(1.0, abs(losses[-1]))
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p1, p2)
