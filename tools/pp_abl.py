#!/usr/bin/env python3
"""Phase-budget ablation of the v14 kernel (conv_pp.hip, tile 117): times one layer with
parts of the 8-phase loop compiled out (KVEDGE_PP_ABL: 1 no MFMA clusters, 2 no fragment
reads, 4 no LDS-DMA staging, 8 no lgkmcnt(0) before the first barrier, 16 no barriers, and
sums of those).  Timing only -- the ablated outputs are wrong.

  for a in 0 1 2 4 6 8 16 22; do KVEDGE_PP_ABL=$a python tools/pp_abl.py --layer s3.c2; done
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAYERS = {  # name: (hw, cin, cout, k, stride)
    "s3.c2": (14, 256, 256, 3, 1), "s4.c2": (7, 512, 512, 3, 1), "s3.c1": (14, 1024, 256, 1, 1),
    "s2.c2": (28, 128, 128, 3, 1), "s3.c2s": (28, 256, 256, 3, 2),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="s3.c2")
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--tile", type=int, default=117)
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops
    from kvedge_amd.ops import ConvSpec

    assert ops.load()
    hw, cin, cout, k, s = LAYERS[a.layer]
    spec = ConvSpec.auto(cin, cout, k, s, k // 2, ops.ACT_RELU)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(a.batch, hw, hw, cin, generator=g).to(torch.bfloat16).cuda()
    w = ops.pack_conv_weight(torch.randn(cout, cin, k, k, generator=g) * 0.05, spec).cuda()
    b = torch.randn(cout, generator=g).cuda()
    Ho, Wo = spec.out_hw(hw, hw)
    y = torch.empty(a.batch, Ho, Wo, cout, dtype=torch.bfloat16, device="cuda")

    def run():
        ops._native().conv(x, w, b, None, y, a.batch, hw, hw, spec.cin_eff, cin, 0, Ho, Wo, cout,
                           k, k, s, k // 2, spec.K, cout, 0, 0, 0, spec.act, spec.mode, a.tile,
                           None)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(10):
            run()
        en.record()
        torch.cuda.synchronize()
        ts.append(st.elapsed_time(en) / 10 * 1e3)
    ts.sort()
    print(f"{a.layer} b{a.batch} tile {a.tile} abl {os.environ.get('KVEDGE_PP_ABL', '0')}: "
          f"{ts[len(ts) // 2]:.1f} us per launch (median of 5 x 10)")


if __name__ == "__main__":
    main()
