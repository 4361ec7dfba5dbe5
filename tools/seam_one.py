#!/usr/bin/env python3
"""Run one v9 seam tile on one ResNet-50 seam shape, for rocprofv3 PMC passes:
  rocprofv3 --kernel-trace --pmc ... -- python3 tools/seam_one.py --shape s3 --tile 7"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--shape", default="s3", choices=["s2", "s2s3", "s3"])
    ap.add_argument("--tile", type=int, default=-1, help="seam tile index (-1: default pick)")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch

    from kvedge_amd import ops

    assert ops.load()
    hw, k3, n1 = {"s2": (28, 128, 128), "s2s3": (28, 128, 256), "s3": (14, 256, 256)}[a.shape]
    B, cout = a.batch, 4 * k3
    g = torch.Generator(device="cuda").manual_seed(0)
    rnd = lambda *s, sc=1.0: (torch.randn(*s, generator=g, device="cuda") * sc).to(torch.bfloat16)  # noqa
    t, r = rnd(B, hw, hw, k3), rnd(B, hw, hw, cout)
    w3, w1 = rnd(cout, k3, sc=(2.0 / k3) ** 0.5), rnd(n1, cout, sc=(2.0 / cout) ** 0.5)
    b3 = torch.randn(cout, generator=g, device="cuda") * 0.1
    b1 = torch.randn(n1, generator=g, device="cuda") * 0.1
    tile = -1 if a.tile < 0 else int(torch.ops.kvedge.conv_num_tiles()) + a.tile
    for _ in range(a.iters):
        ops.conv_tail(t, w3, b3, ops.ACT_RELU, w1, b1, res=r, tile=tile)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
