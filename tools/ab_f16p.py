"""A/B (tuning only): the PPI forward and train step with the projection / g_x GEMMs on the
pre-split f16x3 kernel (gemm_f16p.hip) vs the in-loop split kernel, interleaved in one process
(GATX_F16P toggled between rounds). Prints per-step times, the GEMM spans' mean times and the
max output difference between the two paths.
    python tools/ab_f16p.py [--rounds 5] [--steps 20]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import gatx
    from gatx import data as gd
    from gatx import functional as gf
    from gatx.capture import CapturedStep
    from gatx.config import data_config
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = gatx.GATModel(**data_config["PPI"]).to(dev).eval()
    b = gd.dataset_batch("PPI", 20, graph_seed=42, feature_seed=1)
    x = torch.from_numpy(b.x).to(dev)
    ei = torch.from_numpy(b.edge_index).to(dev)

    def fwd():
        gatx.clear_graph_cache()
        with torch.no_grad():
            return model(x, ei)

    outs, caps = {}, {}
    # (the weight cache is shared by both arms and never cleared: the captured graphs read the
    # cached W_aug and planes by address)
    for arm in ("1", "0"):
        os.environ["GATX_F16P"] = arm
        gf.reset_tuning()
        outs[arm] = fwd().clone()
        caps[arm] = CapturedStep(fwd)
    d = float((outs["1"] - outs["0"]).abs().max())
    print(f"max|out(f16p) - out(in-loop)| = {d:.3e}", flush=True)
    res = {"1": [], "0": []}
    spans = {"1": [], "0": []}
    for _ in range(args.rounds):
        for arm in ("1", "0"):
            os.environ["GATX_F16P"] = arm
            gf.reset_tuning()
            st = caps[arm]
            st()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                st()
            torch.cuda.synchronize()
            res[arm].append((time.perf_counter() - t0) / args.steps * 1e3)
            timer = gf.KernelTimer()
            gf.set_kernel_timer(timer)
            fwd()
            gf.set_kernel_timer(None)
            summ = timer.summary()
            spans[arm].append([t for _, t in summ.get("gemm", [])])
    for arm, name in (("1", "f16p (pre-split weight)"), ("0", "in-loop split")):
        g = [statistics.mean(v) for v in zip(*spans[arm])]
        print(f"{name:26s} fwd {statistics.median(res[arm]):.4f} ms/step (min {min(res[arm]):.4f})"
              f"  projection GEMMs {', '.join(f'{t * 1e3:.1f}' for t in g)} us", flush=True)


if __name__ == "__main__":
    main()
