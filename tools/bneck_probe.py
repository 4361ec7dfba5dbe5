#!/usr/bin/env python3
"""Standalone timing of the v11 fused bottleneck (ops.bottleneck_fused) at a bench slice,
against the same block run unfused (3x3 + conv3 + residual; the bench additionally fuses
conv3 into the next conv1), with debug probes:
  dbg 4: every weight load out of range (zeros) -> the kernel without its weight stream.
  python tools/bneck_probe.py --batch 640
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kvedge_amd import ops  # noqa: E402
from kvedge_amd.ops import ConvSpec  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    torch.cuda._sleep(int(5e7))
    ev = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=640)
    a = ap.parse_args()
    assert ops.load()
    for C, H in ((128, 28), (256, 14)):
        C4, N = 4 * C, a.batch
        g = torch.Generator().manual_seed(0)
        x = torch.relu(torch.randn(N, H, H, C4, generator=g)).to(torch.bfloat16).cuda()
        s1 = ConvSpec.auto(C4, C, 1, 1, 0, ops.ACT_RELU)
        s2 = ConvSpec.auto(C, C, 3, 1, 1, ops.ACT_RELU)
        s3 = ConvSpec.auto(C, C4, 1, 1, 0, ops.ACT_RELU)
        w1 = ops.pack_conv_weight(torch.randn(C, C4, 1, 1, generator=g) * (2.0 / C4) ** 0.5, s1).cuda()
        w2 = ops.pack_conv_weight(torch.randn(C, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5, s2).cuda()
        w3 = ops.pack_conv_weight(torch.randn(C4, C, 1, 1, generator=g) * (1.0 / C) ** 0.5, s3).cuda()
        b1, b2, b3 = (torch.zeros(n, device="cuda") for n in (C, C, C4))
        frag = tuple(ops.mfma_frag_major(w) for w in (w1, w2, w3))
        y = torch.empty_like(x)
        z1 = torch.empty(N, H, H, C, dtype=torch.bfloat16, device="cuda")
        z2 = torch.empty_like(z1)
        res = {}
        # dbg 1 / 2: stop after phase 1 / 2 (dumping z1 / z2); +4: no weight traffic
        for dbg in (0, 4, 1, 5, 2, 6):
            res[f"fused dbg{dbg}"] = timeit(lambda: ops.bottleneck_fused(
                x, w1, b1, w2, b2, w3, b3, out=y, frag=frag, _dbg=dbg))
        res["unfused conv1"] = timeit(lambda: ops.conv2d(x, s1, w1, b1, out=z1))
        res["unfused 3x3"] = timeit(lambda: ops.conv2d(z1, s2, w2, b2, out=z2))
        res["unfused conv3+res"] = timeit(lambda: ops.conv2d(z2, s3, w3, b3, res=x, out=y))
        flops = 2.0 * N * H * H * 17 * C * C
        print(f"C{C} {H}x{H} b{N}: " + ", ".join(f"{k} {v:.1f} us" for k, v in res.items()) +
              f"; fused {flops / res['fused dbg0'] / 1e9:.2f} PF/s", flush=True)


if __name__ == "__main__":
    main()
