"""Diagnostic: why the PPI-20 train step's L2 weight-gradient GEMM (gemm_f16rc) falls back to x3
with tuning side_stream=0. Intercepts gatx_gemm_wgrad's operands and reports non-finite / out-of-
range entries of G_aug (incl. the per-head padding columns F..Fp) and of x per K-slice."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gat-pytorch_amd"))
import torch  # noqa: E402
import gatx  # noqa: E402
from gatx import functional as gf, tuning, _lib  # noqa: E402
from gatx import data as gd  # noqa: E402
from gatx.config import data_config  # noqa: E402

side = int(sys.argv[1]) if len(sys.argv) > 1 else 0
tuning.set(side_stream=side)
reg = {}


class TP:
    def __getattr__(self, n):
        return getattr(torch, n)

    def empty(self, *a, **k):
        t = torch.empty(*a, **k)
        reg[t.data_ptr()] = t
        return t


gf.torch = TP()
orig_call = gf.call
fb = torch.zeros(1, dtype=torch.int64, device="cuda")


captured = []
CAP = len(sys.argv) > 2 and sys.argv[2] == "cap"


def inspect(KC, Fin, N, ldg, G, x, cm):
        print(f"wgrad KC={KC} Fin={Fin} N={N} ldg={ldg} G={G is not None} x={x is not None}")
        if G is not None:
            Gv = G.view(-1)[:N * ldg].view(N, ldg)[:, :KC]
            print("  G_aug nonfinite:", int((~torch.isfinite(Gv)).sum()), " max|G|:", float(Gv.abs().nan_to_num(0).max()))
            if KC == 756:
                for h in range(6):
                    pad = Gv[:, h * 124 + 121: h * 124 + 124]
                    print(f"  head {h} pad cols: nonfinite {int((~torch.isfinite(pad)).sum())} max {float(pad.abs().nan_to_num(0).max()):.3e}")
        if cm is not None:
            print("  colmax nonfinite:", int((~torch.isfinite(cm[:KC])).sum()), "max", float(cm[:KC].nan_to_num(0).max()), "min", float(cm[:KC].min()))
        if x is not None:
            xv = x[:N, :Fin]
            print("  x nonfinite:", int((~torch.isfinite(xv)).sum()), "max", float(xv.abs().max()))
            for s0 in range(0, N, 2138):
                m = xv[s0:s0 + 2138].abs().max(0).values
                bad = ((m > 0) & (m < 2 ** -13)) | (m > 65504)
                if bad.any():
                    print(f"  slice {s0}: {int(bad.sum())} bad cols, e.g. {m[bad][:4].tolist()}")
                    break


def call(name, *args):
    if name == "gatx_gemm_wgrad" and CAP and torch.cuda.is_current_stream_capturing():
        KC, Fin, N, Gp, ldg, xp, _, cmp = args[:8]
        captured.append((KC, Fin, N, ldg, reg.get(Gp), reg.get(xp), reg.get(cmp), Gp, xp, cmp))
        return orig_call(name, *args)
    if name == "gatx_gemm_wgrad":
        KC, Fin, N, Gp, ldg, xp, _, cmp = args[:8]
        G, x, cm = reg.get(Gp), reg.get(xp), reg.get(cmp)
        torch.cuda.synchronize()
        _lib.call("gatx_gemm_fallback_read", _lib.ptr(fb), 1, _lib.stream())
        torch.cuda.synchronize()
        print(f"wgrad KC={KC} Fin={Fin} N={N} ldg={ldg} G={G is not None} x={x is not None}")
        if G is not None:
            Gv = G.view(-1)[:N * ldg].view(N, ldg)[:, :KC]
            print("  G_aug nonfinite:", int((~torch.isfinite(Gv)).sum()), " max|G|:", float(Gv.abs().nan_to_num(0).max()))
            for h in range(6):
                pad = Gv[:, h * 124 + 121: h * 124 + 124]
                print(f"  head {h} pad cols: nonfinite {int((~torch.isfinite(pad)).sum())} max {float(pad.abs().nan_to_num(0).max()):.3e}")
        if cm is not None:
            print("  colmax nonfinite:", int((~torch.isfinite(cm[:KC])).sum()), "max", float(cm[:KC].nan_to_num(0).max()))
        if x is not None:
            xv = x[:N, :Fin]
            print("  x nonfinite:", int((~torch.isfinite(xv)).sum()), "max", float(xv.abs().max()))
            for s0 in range(0, N, 2138):
                m = xv[s0:s0 + 2138].abs().max(0).values
                bad = ((m > 0) & (m < 2 ** -13)) | (m > 65504)
                if bad.any():
                    print(f"  slice {s0}: {int(bad.sum())} bad cols, e.g. {m[bad][:4].tolist()}")
                    break
        orig_call(name, *args)
        torch.cuda.synchronize()
        _lib.call("gatx_gemm_fallback_read", _lib.ptr(fb), 1, _lib.stream())
        torch.cuda.synchronize()
        print("  fallback tiles in this launch:", int(fb.item()))
        return
    return orig_call(name, *args)


gf.call = call
dev = torch.device("cuda")
cfg = dict(data_config["PPI"])
torch.manual_seed(0)
model = gatx.GATModel(**cfg).to(dev).train()
b = gd.dataset_batch("PPI", 20, graph_seed=42, feature_seed=1)
x = torch.from_numpy(b.x).to(dev)
ei = torch.from_numpy(b.edge_index).to(dev)
y = (torch.rand(b.num_nodes, 121, device=dev) > 0.5).float()
from gatx.losses import BCEWithLogitsLoss  # noqa: E402
opt = torch.optim.Adam(model.parameters(), lr=0.005, capturable=CAP, fused=True)
from gatx.graph import expect_num_edges, graph_cache
expect_num_edges(ei, b.num_nodes, True, graph_cache.get(ei, b.num_nodes, True).num_edges)
one = torch.ones((), device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    gatx.clear_graph_cache()
    out, ei2, atts = model.forward_and_return_attention(x, ei)
    loss = BCEWithLogitsLoss()(out, y)
    model.calc_attention_norm(ei2, atts)
    loss.backward(one)
    opt.step()
    return out


if not CAP:
    for it in range(2):
        print("== step", it)
        step()
else:
    from gatx.capture import CapturedStep
    st = CapturedStep(step)
    print("captured wgrad calls:", [(c[0], c[4] is not None, c[5] is not None, c[6] is not None) for c in captured])
    for it in range(3):
        _lib.call("gatx_gemm_fallback_read", _lib.ptr(fb), 1, _lib.stream())
        st()
        torch.cuda.synchronize()
        _lib.call("gatx_gemm_fallback_read", _lib.ptr(fb), 1, _lib.stream())
        torch.cuda.synchronize()
        print("replay", it, "fallback tiles:", int(fb.item()))
    for c in captured:
        inspect(*c[:7])
torch.cuda.synchronize()
