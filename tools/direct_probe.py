#!/usr/bin/env python3
"""Time one conv shape on one tile (default: ResNet-50 layer1 3x3 on the v4 direct tile)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="640,56,56,64,64,3,1")  # N,H,W,cin,cout,k,stride
    ap.add_argument("--tile", type=int, default=34)
    ap.add_argument("--act", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops
    from kvedge_amd.ops import ConvSpec

    assert ops.load()
    N, H, W, ci, co, k, s = (int(v) for v in a.shape.split(","))
    spec = ConvSpec.auto(ci, co, k, s, k // 2, a.act)
    x = (torch.randn(N, H, W, ci, device="cuda") * 0.5).to(torch.bfloat16)
    w = ops.pack_conv_weight(torch.randn(co, ci, k, k) * 0.05, spec).cuda()
    b = torch.randn(co, device="cuda")
    out = ops.conv2d(x, spec, w, b, tile=a.tile)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.reps):
        ops.conv2d(x, spec, w, b, out=out, tile=a.tile)
    en.record()
    torch.cuda.synchronize()
    us = st.elapsed_time(en) / a.reps * 1e3
    Ho, Wo = spec.out_hw(H, W)
    fl = 2.0 * N * Ho * Wo * co * ci * k * k
    by = 2.0 * (N * H * W * ci + N * Ho * Wo * co)
    print(f"{a.shape} tile {a.tile}: {us:.1f} us  {fl / us / 1e6:.0f} TF/s  {by / us / 1e3:.0f} GB/s")


if __name__ == "__main__":
    main()
