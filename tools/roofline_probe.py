#!/usr/bin/env python3
"""Practical ceilings on this MI355X, measured (not datasheet): HBM bandwidth for the
access mixes our layers have (read-only, 1R1W copy, 2R1W add) and hipBLASLt bf16 GEMM
throughput on the GEMM shapes of ResNet-50's convs (implicit-GEMM M x N x K).
Used to judge how far each kernel in profiles/*forward*.md is from speed of light."""
import json
import sys

import torch


def _time(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    out = {"bw_TBps": {}, "gemm_TFLOPs": {}}
    n = 400 * 2**20 // 2  # 400 MiB of bf16
    a = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    c = torch.empty_like(a)
    nb = n * 2
    out["bw_TBps"]["read (sum)"] = nb / _time(lambda: a.sum()) / 1e12
    out["bw_TBps"]["write (fill)"] = nb / _time(lambda: c.fill_(1.0)) / 1e12
    out["bw_TBps"]["1R1W (copy)"] = 2 * nb / _time(lambda: c.copy_(a)) / 1e12
    out["bw_TBps"]["2R1W (add)"] = 3 * nb / _time(lambda: torch.add(a, b, out=c)) / 1e12
    del a, b, c
    if "--bw-only" in sys.argv:
        json.dump(out, sys.stdout, indent=1)
        return
    shapes = {  # name: (M, N, K)
        "s1 3x3 64->64 (M=802816)": (802816, 64, 576),
        "s2 3x3 128->128": (200704, 128, 1152),
        "s3 3x3 256->256": (50176, 256, 2304),
        "s4 3x3 512->512": (12544, 512, 4608),
        "s3 c1 1024->256": (50176, 256, 1024),
        "s4 c1 2048->512": (12544, 512, 2048),
        "square 8192": (8192, 8192, 8192),
    }
    for name, (M, N, K) in shapes.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        t = _time(lambda: x @ w)
        out["gemm_TFLOPs"][name] = 2 * M * N * K / t / 1e12
        del x, w
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
