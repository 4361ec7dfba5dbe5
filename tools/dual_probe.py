#!/usr/bin/env python3
"""Time the fused conv3 + downsample (dual-source) GEMMs of ResNet-50 stages 2-4 on chosen
tiles (tools/tile_probe.py covers single-source convs only).
  python tools/dual_probe.py --batch 640 --tiles 30,63,64,65"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tiles", default="30")
    ap.add_argument("--only", default="", help="comma list of layer names (s2.dual, ...)")
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops

    assert ops.load()
    B = a.batch
    tiles = [int(t) for t in a.tiles.split(",")]
    # (name, Ho, K1 (conv2 out ch), K2 (block input ch), Cout), stride 2 downsample
    layers = [("s2.dual", 28, 128, 256, 512), ("s3.dual", 14, 256, 512, 1024),
              ("s4.dual", 7, 512, 1024, 2048)]
    if a.only:
        layers = [l for l in layers if l[0] in a.only.split(",")]
    print("| layer | " + " | ".join(str(t) for t in tiles) + " | GB |")
    print("|---" * (len(tiles) + 2) + "|")
    for name, ho, k1, k2, co in layers:
        x1 = torch.randn(B, ho, ho, k1, device="cuda").to(torch.bfloat16)
        x2 = torch.randn(B, 2 * ho, 2 * ho, k2, device="cuda").to(torch.bfloat16)
        w = (torch.randn(co, k1 + k2, device="cuda") * 0.05).to(torch.bfloat16)
        b = torch.randn(co, device="cuda")
        byts = 2.0 * B * ho * ho * (k1 + k2 + co)
        cells = []
        for t in tiles:
            try:
                fn = lambda: ops.conv_dual(x1, x2, w, b, ops.ACT_RELU, 2, tile=t)  # noqa: E731
                for _ in range(3):
                    fn()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                st.record()
                for _ in range(a.iters):
                    fn()
                en.record()
                torch.cuda.synchronize()
                cells.append(f"{st.elapsed_time(en) / a.iters * 1e3:.1f}")
            except RuntimeError:
                cells.append("-")
        print(f"| {name} | " + " | ".join(cells) + f" | {byts / 1e9:.3f} |", flush=True)


if __name__ == "__main__":
    main()
