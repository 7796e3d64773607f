"""hipGraph capture of whole gatx steps (small batches are launch-bound).

A GATModel forward is ~10 launches per layer plus the graph build; a training step ~40 per
layer. At PATTERN's batch of 8 graphs (951 nodes) or PPI's reference batch of 2 the kernels are a
few microseconds each, so the host's per-launch Python + ctypes cost decides the step time
(SURVEY.md §7 "Hard parts"). Every gatx entry point is capturable by construction: launches go to
torch's current stream, nothing allocates outside torch's caching allocator, nothing synchronises
(|edge_index'| stays on the device, the dropout seed is drawn by torch's generator on the device).
So a whole step — graph build, forward, and for training backward + optimizer — is captured once
and replayed as one hipGraph launch.

    step = CapturedStep(lambda: model(x, edge_index))   # x / edge_index: static device tensors
    out = step()                                          # replay: refill x in place to change it

Rules (torch.cuda.graph's): inputs are read from the same addresses every replay (copy new data
into them in place), outputs are overwritten by the next replay, and the step must not read a
device value on the host (a layer asked for its attention weights reads |edge_index'|: capture
such steps only when that read happened before capture, or run them eagerly). Optimizers inside
a captured training step need capturable=True (e.g. torch.optim.Adam(..., capturable=True)).
"""
from __future__ import annotations

import torch


class CapturedStep:
    """Capture `fn()` into a hipGraph after `warmup` eager runs on a side stream (which settle the
    caching allocator and every lazy init); each call replays it and returns the static output.

    The warm-ups and the capture run on the SAME side stream (`self.stream`): a training step's
    autograd graph can outlive the step (GATLayer keeps its last alpha, as the reference's
    `normalised_attention_coeffs` does, and that tensor holds the graph), and with it the
    parameters' AccumulateGrad nodes, which remember the stream they were created on. Capturing
    on another stream than the warm-ups would make the captured backward accumulate across
    streams (torch warns: extra synchronisation, and it can break capture). `eager()` runs the
    step outside the graph on that same stream (e.g. HIP-event-instrumented steps)."""

    def __init__(self, fn, warmup: int = 2, pool=None):
        self.fn = fn
        self.stream = s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=pool, stream=s):
            self.out = fn()

    def __call__(self):
        self.graph.replay()
        return self.out

    def eager(self):
        """One un-captured run of the step on the capture stream, ordered after everything
        already enqueued on the current stream (and the current stream after it)."""
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            out = self.fn()
        cur.wait_stream(self.stream)
        return out

    def reset(self):
        self.graph.reset()
