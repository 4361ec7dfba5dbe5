#!/usr/bin/env python3
"""Time (or profile under rocprofv3) ONE conv shape on chosen tiles.

  python tools/conv_probe.py --shape 192,80,80,64,128,3,1 --act silu --tiles 54,55,56,57
  rocprofv3 --kernel-trace --pmc ... -- python3 tools/conv_probe.py --shape ... --tiles 55 --iters 3
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", required=True, help="N,H,W,cin,cout,k,stride")
    ap.add_argument("--act", default="silu", choices=["none", "relu", "silu"])
    ap.add_argument("--res", action="store_true")
    ap.add_argument("--tiles", default="-1")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()

    import torch
    from kvedge_amd import ops

    assert ops.load()
    N, H, W, cin, cout, k, s = (int(v) for v in a.shape.split(","))
    act = {"none": ops.ACT_NONE, "relu": ops.ACT_RELU, "silu": ops.ACT_SILU}[a.act]
    if a.res:
        act |= ops.RES_AFTER_ACT
    spec = ops.ConvSpec.auto(cin, cout, k, s, k // 2, act)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, W, cin, generator=g).to(torch.bfloat16).cuda()
    w = ops.pack_conv_weight(torch.randn(cout, cin, k, k, generator=g) * 0.05, spec).cuda()
    b = torch.randn(cout, generator=g).cuda()
    Ho, Wo = spec.out_hw(H, W)
    res = torch.randn(N, Ho, Wo, cout, generator=g).to(torch.bfloat16).cuda() if a.res else None
    out = torch.empty(N, Ho, Wo, cout, dtype=torch.bfloat16, device="cuda")
    flops = 2.0 * N * Ho * Wo * cout * k * k * cin
    for t in (int(v) for v in a.tiles.split(",")):
        try:
            ops.conv2d(x, spec, w, b, res=res, out=out, tile=t)
        except RuntimeError as e:
            print(f"tile {t}: not valid ({str(e)[:60]})")
            continue
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(5e6))
        e0.record()
        for _ in range(a.iters):
            ops.conv2d(x, spec, w, b, res=res, out=out, tile=t)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(f"tile {t}: {us:.1f} us  {flops / us / 1e9:.3f} PF/s", flush=True)


if __name__ == "__main__":
    main()
