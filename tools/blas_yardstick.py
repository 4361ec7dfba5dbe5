#!/usr/bin/env python3
"""hipBLASLt yard-stick for the ResNet-50 1x1 layers (b640): torch.mm bf16 on the same
GEMM shapes (no epilogue, no residual) -- how far the hand-written conv GEMMs sit from
the vendor library on plain GEMM work."""
import torch

SHAPES = {  # name: (M, K, N)
    "s2.c1 512->128": (501760, 512, 128),
    "s2.dual 384->512": (501760, 384, 512),
    "s3.c1 1024->256": (125440, 1024, 256),
    "s3.c3 256->1024": (125440, 256, 1024),
    "s3.dual 768->1024": (125440, 768, 1024),
    "s4.c1 2048->512": (31360, 2048, 512),
    "s4.c3 512->2048": (31360, 512, 2048),
    "s3.c2 as gemm 2304->256": (125440, 2304, 256),
}


def main():
    print("| layer | M | K | N | torch.mm us | TF/s |")
    print("|---|---|---|---|---|---|")
    for name, (M, K, N) in SHAPES.items():
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            torch.mm(a, b)
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        st.record()
        for _ in range(it):
            torch.mm(a, b)
        en.record()
        torch.cuda.synchronize()
        us = st.elapsed_time(en) / it * 1e3
        print(f"| {name} | {M} | {K} | {N} | {us:.1f} | {2 * M * K * N / us / 1e6:.0f} |",
              flush=True)


if __name__ == "__main__":
    main()
