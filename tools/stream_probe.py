"""Probe: does splitting one ResNet-50 step into S batch slices on S HIP streams (one
hipGraph with S parallel branches) overlap the compute-bound 3x3 convs of one slice with
the HBM-bound 1x1 / tail kernels of another?

Each config is S:stagger.  stagger -2: no dependency between the branches (lock-step);
-1: slice i+1 starts when slice i has finished its stem; k >= 0: when slice i has finished
bottleneck k -- the branches then run phase-shifted.  Measured (profiles/r2_v17_stream_probe.jsonl):
two slices in lock-step win; 3-4 slices and every phase shift lose.

  python tools/stream_probe.py --batch 1280 --configs 1:-2,2:-2,2:-1,2:2,2:6
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from kvedge_amd import ops  # noqa: E402
from kvedge_amd.engine.autotune import autotune  # noqa: E402
from kvedge_amd.models.resnet import KvResNet50  # noqa: E402


def slice_forward(model, frames, evt=None, at=-1):
    """One slice: stem+pool from raw frames, the bottlenecks (fused tails), head.
    Records ``evt`` after bottleneck ``at`` (at = -1: after the stem)."""
    x = model.stem_and_pool(frames, frames_in=True)
    if evt is not None and at < 0:
        evt.record()
    t1 = None
    blocks = model.blocks
    for i, b in enumerate(blocks):
        nxt = blocks[i + 1] if i + 1 < len(blocks) else None
        if nxt is not None and b.can_tail(nxt):
            x, t1 = b.call_tail(x, nxt, t1=t1)
        else:
            x, t1 = b(x, t1=t1), None
        if evt is not None and i == at:
            evt.record()
    B = x.shape[0]
    pooled = ops.global_avgpool(x).view(B, 1, 1, 2048)
    lg = model.fc(pooled).view(B, model.num_classes)
    return ops.softmax_rows(lg)


def make_step(model, frames, S, stagger):
    B = frames.shape[0]
    per = B // S
    streams = [torch.cuda.Stream() for _ in range(S)]

    def step():
        cur = torch.cuda.current_stream()
        outs = []
        prev = None
        for i, s in enumerate(streams):
            s.wait_stream(cur)
            if prev is not None:
                s.wait_event(prev)
            evt = torch.cuda.Event() if (stagger >= -1 and i + 1 < S) else None
            with torch.cuda.stream(s):
                outs.append(slice_forward(model, frames[i * per:(i + 1) * per], evt,
                                          stagger))
            prev = evt if stagger >= -1 else None
        for s in streams:
            cur.wait_stream(s)
        return outs
    return step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1280)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--configs", default="1:-2,2:-2,2:-1,2:2,2:6")
    ap.add_argument("--eager", action="store_true")
    a = ap.parse_args()
    assert ops.load()
    model = KvResNet50.build(seed=0, device="cuda")
    frames = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device="cuda")
    tuned_for = None
    for cfg in a.configs.split(","):
        S, stagger = (int(v) for v in cfg.split(":"))
        per = a.batch // S
        if tuned_for != per:
            autotune(lambda f: slice_forward(model, f), frames[:per])
            tuned_for = per
        step = make_step(model, frames, S, stagger)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        run = step
        if not a.eager:
            g = torch.cuda.CUDAGraph()
            s0 = torch.cuda.Stream()
            s0.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s0):
                step()
            torch.cuda.current_stream().wait_stream(s0)
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                step()
            run = g.replay
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"batch": a.batch, "streams": S, "stagger": stagger,
                          "graph": not a.eager, "ms_per_step": round(dt * 1e3, 3),
                          "img_s": round(a.batch / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
