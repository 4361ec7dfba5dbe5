#!/usr/bin/env python3
"""Fused layer-1 bottleneck body (ops.conv_block) vs the two-kernel path it replaces
(v4 direct 3x3 + v3 fused tail) on the ResNet-50 stage-1 shapes at one batch.  Times with
HIP events over --iters launches (random post-ReLU inputs), reports us and HBM GB/s of the
compulsory bytes (t + residual | x2 + y + z)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    from kvedge_amd import ops
    from kvedge_amd.ops import ConvSpec

    assert ops.load()
    B, H, W = a.batch, 56, 56
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(torch.bfloat16)

    def timeit(fn):
        for _ in range(3):
            fn()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        st.record()
        for _ in range(a.iters):
            fn()
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / a.iters * 1e3

    spec2 = ConvSpec.auto(64, 64, 3, 1, 1, ops.ACT_RELU)
    direct_tile = 54  # v4 tile 0 (VGPR prefetch); tests/test_kernels_gpu.py DIRECT0
    print("| form | fused us | direct + tail us | saved | fused GB/s |")
    print("|---|---|---|---|---|")
    for name, dual, nt in (("dual (block 0)", True, 64), ("res nt64 (block 1)", False, 64),
                           ("res nt128 (block 2)", False, 128)):
        t = rnd(B, H, W, 64).relu()
        w2, b2 = rnd(64, 576, scale=0.06), torch.randn(64, device=dev) * 0.1
        w3 = rnd(256, 128 if dual else 64, scale=0.12)
        b3 = torch.randn(256, device=dev) * 0.1
        w1, b1 = rnd(nt, 256, scale=0.09), torch.randn(nt, device=dev) * 0.1
        extra = rnd(B, H, W, 64 if dual else 256)
        y = torch.empty(B, H, W, 256, device=dev, dtype=torch.bfloat16)
        z = torch.empty(B, H, W, nt, device=dev, dtype=torch.bfloat16)
        c2 = torch.empty(B, H, W, 64, device=dev, dtype=torch.bfloat16)
        kw = {"x2": extra} if dual else {"res": extra}

        def fused():
            ops.conv_block(t, w2, b2, w3, b3, w1, b1, out=y, z=z, **kw)

        def unfused():
            ops.conv2d(t, spec2, w2, b2, out=c2, tile=direct_tile)
            if dual:
                ops.conv_tail(c2, w3, b3, ops.ACT_RELU, w1, b1, x2=extra, stride2=1, out=y, z=z)
            else:
                ops.conv_tail(c2, w3, b3, ops.ACT_RELU, w1, b1, res=extra, out=y, z=z)

        tf, tu = timeit(fused), timeit(unfused)
        byts = B * H * W * 2 * (64 + (64 if dual else 256) + 256 + nt)
        print(f"| {name} | {tf:.1f} | {tu:.1f} | {tu - tf:.1f} | {byts / tf / 1e3:.0f} |", flush=True)


if __name__ == "__main__":
    main()
