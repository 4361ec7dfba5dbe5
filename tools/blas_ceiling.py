#!/usr/bin/env python3
"""Library ceiling for the ResNet-50 GEMM shapes: torch.matmul (hipBLASLt on ROCm) on the
plain [M, K] x [K, N] bf16 GEMM of each conv at batch --batch, vs our kernel's time from a
roofline table.  The 3x3 rows are priced as their im2col GEMM (K = 9 Cin) with the A matrix
already materialised -- a bound our implicit GEMM does not get for free (it gathers the taps).

  python tools/blas_ceiling.py --batch 640 > gpurun_out/blas_ceiling.md
"""
import argparse

import torch

SHAPES = [  # (name, M per image, K, N)
    ("s1 1x1 64>64", 56 * 56, 64, 64),
    ("s1 3x3 64>64", 56 * 56, 576, 64),
    ("s1 1x1 64>256", 56 * 56, 64, 256),
    ("s2 1x1 512>128", 28 * 28, 512, 128),
    ("s2 3x3 128>128", 28 * 28, 1152, 128),
    ("s2 1x1 128>512", 28 * 28, 128, 512),
    ("s3 1x1 1024>256", 14 * 14, 1024, 256),
    ("s3 3x3 256>256", 14 * 14, 2304, 256),
    ("s3 1x1 256>1024", 14 * 14, 256, 1024),
    ("s3 dual 768>1024", 14 * 14, 768, 1024),
    ("s4 1x1 2048>512", 7 * 7, 2048, 512),
    ("s4 3x3 512>512", 7 * 7, 4608, 512),
    ("s4 1x1 512>2048", 7 * 7, 512, 2048),
    ("s4 dual 1536>2048", 7 * 7, 1536, 2048),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    print(f"# torch.matmul (hipBLASLt) bf16 on the ResNet-50 GEMM shapes, batch {a.batch}\n")
    print("| layer | M | K | N | us | PF/s | TB/s (A+B+C once) |")
    print("|---|---|---|---|---|---|---|")
    for name, mpi, k, n in SHAPES:
        m = mpi * a.batch
        x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
        y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(x, w, out=y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            torch.matmul(x, w, out=y)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        fl = 2.0 * m * k * n
        by = 2.0 * (m * k + k * n + m * n)
        print(f"| {name} | {m} | {k} | {n} | {us:.1f} | {fl / us / 1e9:.3f} | {by / us / 1e6:.2f} |",
              flush=True)
        del x, w, y


if __name__ == "__main__":
    main()
