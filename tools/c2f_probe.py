#!/usr/bin/env python3
"""Standalone timing of the v13 fused C2f kernel (ops.c2f16) against its compulsory traffic
(x read + y written once) and the four-launch block it replaces, per strip height S.

  python tools/c2f_probe.py --batch 256 --strips 40,20,8
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hw", type=int, default=160)
    ap.add_argument("--strips", default="40,20,8")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--diags", default="", help="KVEDGE_C2F_DIAG values to time at the first S "
                    "(1 identity act, 2 no x loads, 4 no y stores, 8 y via LDS staging)")
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops
    from kvedge_amd.models.yolov8 import C2f, DC2f

    assert ops.load()
    torch.manual_seed(0)
    blk = DC2f(C2f(32, 32, 1, True).eval(), "cuda")
    b1, b2, _ = blk.m[0]
    x = torch.randn(a.batch, a.hw, a.hw, 32, device="cuda").to(torch.bfloat16)
    y = torch.empty_like(x)
    byts = 2 * x.numel() * 2

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(3):
            g.replay()
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / (3 * a.iters) * 1e3

    print(f"c2f16 b{a.batch} @{a.hw}: compulsory {byts / 1e6:.0f} MB")
    for S in [int(s) for s in a.strips.split(",")]:
        us = timeit(lambda: ops.c2f16(x, blk.cv1.w, blk.cv1.b, b1.w, b1.b, b2.w, b2.b,
                                      blk.cv2.w, blk.cv2.b, out=y, S=S))
        print(f"  fused S={S}: {us:.1f} us  {byts / us / 1e3:.0f} GB/s", flush=True)
    S0 = int(a.strips.split(",")[0])
    for d in [int(v) for v in a.diags.split(",") if v]:
        os.environ["KVEDGE_C2F_DIAG"] = str(d)
        us = timeit(lambda: ops.c2f16(x, blk.cv1.w, blk.cv1.b, b1.w, b1.b, b2.w, b2.b,
                                      blk.cv2.w, blk.cv2.b, out=y, S=S0))
        print(f"  fused S={S0} diag={d}: {us:.1f} us", flush=True)
    os.environ.pop("KVEDGE_C2F_DIAG", None)
    ops.C2F_ENABLED = False
    us = timeit(lambda: blk(x, out=y))
    print(f"  four launches: {us:.1f} us", flush=True)
    z = torch.empty_like(x)
    us = timeit(lambda: z.copy_(x))
    print(f"  torch copy of x (same bytes): {us:.1f} us  {byts / us / 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
