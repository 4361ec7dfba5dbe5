#!/usr/bin/env python3
"""Comparison point: the same ResNet-50 through stock PyTorch-ROCm (MIOpen/hipBLASLt),
bf16 channels_last, BN folded is NOT applied (eval-mode BN, as a user would run it),
optionally captured in a CUDA(hip)Graph.  Prints one JSON line.  Not the headline
metric -- only the yard-stick our hand-written kernels must beat."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    import torch
    from kvedge_amd.models.resnet import init_resnet50

    m = init_resnet50(0, calibrate=False).cuda().to(torch.bfloat16).to(
        memory_format=torch.channels_last).eval()
    x = torch.randn(a.batch, 3, 224, 224, device="cuda", dtype=torch.bfloat16).to(
        memory_format=torch.channels_last)

    def step():
        with torch.no_grad():
            return torch.softmax(m(x).float(), 1)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    run = step
    if a.graph:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            step()
        run = g.replay
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"impl": "torch-miopen", "graph": a.graph, "batch": a.batch,
                      "images_per_s": round(a.batch * a.steps / dt, 1),
                      "ms_per_step": round(dt / a.steps * 1e3, 3)}))


if __name__ == "__main__":
    main()
