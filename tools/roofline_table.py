#!/usr/bin/env python3
"""Per-layer roofline table of one ResNet-50 step from a rocprofv3 kernel trace.

Input: the kernel-trace CSV of `tools/profile_forward.py` (ResNet-50, default deployed path:
frames-in stem+pool, stage-1 fused tails, direct / LDS-DMA / streaming convs, fused
downsample GEMMs).  The step's kernel sequence is fixed, so kernel i of the last replayed
step is matched to layer i of the list below, which carries each launch's compulsory HBM
bytes (inputs read once, outputs written once, strided downsample sources counted at the
pixels they read) and its model FLOPs (2 x MACs of the real convolution; the s2d stem at
its 7x7x3 taps).  Floors: HBM at --hbm TB/s, MFMA at --peak PF/s; 'floor' is the larger,
'eff' = floor / measured.

  python tools/roofline_table.py gpurun_out/fwd/fwd_kernel_trace.csv --batch 640
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def layers(B, seam=False):
    """[(name, kernel-name fragment, bytes, flops)] in launch order for batch B."""
    MB = 1e-6
    L = []

    def t(n, hw, c):  # bf16 activation bytes
        return n * hw * hw * c * 2

    def gemm(m, k, n):
        return 2.0 * m * k * n

    L.append(("frames (synth)", "synth", B * 224 * 224 * 3, 0))
    L.append(("step counter", "bump", 8, 0))
    L.append(("stem 7x7/2 + maxpool (frames in)", "stem",
              B * 224 * 224 * 3 + t(B, 56, 64), gemm(B * 112 * 112, 147, 64)))
    m1 = B * 56 * 56
    L.append(("s1.b0 conv1 64>64", "conv", 2 * t(B, 56, 64), gemm(m1, 64, 64)))
    # three stage-1 blocks: direct 3x3, then the fused tail (conv3 + residual|downsample +
    # next block's conv1)
    for b, (dual, nt) in enumerate(((True, 64), (False, 64), (False, 128))):
        L.append((f"s1.b{b} conv2 3x3 64>64", "conv", 2 * t(B, 56, 64), gemm(m1, 576, 64)))
        src = t(B, 56, 64) if dual else t(B, 56, 256)
        L.append((f"s1.b{b} tail conv3{'+down' if dual else '+res'} -> next conv1 ({nt})", "conv",
                  t(B, 56, 64) + src + t(B, 56, 256) + t(B, 56, nt),
                  gemm(m1, 64 + (64 if dual else 0), 256) + gemm(m1, 256, nt)))
    # stages 2-4; with seam=True the v9 seam kernel (conv_seam.hip) runs a plain
    # conv3 + residual together with the NEXT block's conv1 (stages 2, 2->3, 3, 3->4)
    from kvedge_amd.ops import SEAM_SHAPES as seam_shapes
    stages = [  # (stage, hw_in, hw, width, blocks)
        (2, 56, 28, 128, 4), (3, 28, 14, 256, 6), (4, 14, 7, 512, 3)]
    pending_c1 = 128  # conv1 of the next block already computed (stage-1 tail, or a seam)
    for si, (st, hwi, hw, wd, nb) in enumerate(stages):
        m = B * hw * hw
        cout = 4 * wd
        for b in range(nb):
            cin = (2 * wd if st > 2 else 256) if b == 0 else cout
            hin = hwi if b == 0 else hw
            if pending_c1 is None:
                L.append((f"s{st}.b{b} conv1 {cin}>{wd}" + (f" ({hin}x{hin})" if b == 0 and st > 2 else ""),
                          "conv", t(B, hin, cin) + t(B, hin, wd), gemm(B * hin * hin, cin, wd)))
            pending_c1 = None
            if b == 0:
                L.append((f"s{st}.b0 conv2 3x3/2 {wd}>{wd}", "conv", t(B, hin, wd) + t(B, hw, wd),
                          gemm(m, 9 * wd, wd)))
                L.append((f"s{st}.b0 conv3+down (dual) {wd + cin}>{cout}", "conv",
                          t(B, hw, wd) + t(B, hw, cin) + t(B, hw, cout), gemm(m, wd + cin, cout)))
                continue
            L.append((f"s{st}.b{b} conv2 3x3 {wd}>{wd}", "conv", 2 * t(B, hw, wd), gemm(m, 9 * wd, wd)))
            last = b == nb - 1
            nt = (2 * wd if st < 4 else None) if last else wd
            if seam and nt is not None and (wd, cout, nt) in seam_shapes:
                L.append((f"s{st}.b{b} seam conv3+res -> next conv1 ({nt})", "seam",
                          t(B, hw, wd) + 2 * t(B, hw, cout) + t(B, hw, nt),
                          gemm(m, wd, cout) + gemm(m, cout, nt)))
                pending_c1 = nt
            else:
                L.append((f"s{st}.b{b} conv3 {wd}>{cout} +res", "conv", t(B, hw, wd) + 2 * t(B, hw, cout),
                          gemm(m, wd, cout)))
    L.append(("global avgpool", "avgpool", t(B, 7, 2048) + B * 2048 * 2, 0))
    L.append(("fc 2048>1000", "conv", B * 2048 * 2 + B * 1000 * 2 + 2048 * 1000 * 2,
              gemm(B, 2048, 1000)))
    L.append(("softmax + top1", "softmax", B * 1000 * 2 + B * 1000 * 4, 0))
    del MB
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--hbm", type=float, default=6.0, help="HBM floor, TB/s")
    ap.add_argument("--peak", type=float, default=2.5, help="dense bf16 MFMA floor, PF/s")
    ap.add_argument("--seam", type=int, default=None,
                    help="1/0: the trace does / does not use the v9 seam kernel (default: detect)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seam = a.seam if a.seam is not None else any("seam" in r["Kernel_Name"] for r in rows)
    L = layers(a.batch, seam)
    # the step-counter bump is its own launch only in traces older than the in-kernel bump
    if not any("bump_kernel" in r["Kernel_Name"] for r in rows):
        L = [x for x in L if x[1] != "bump"]
    starts = [i for i, r in enumerate(rows) if "synth_dev" in r["Kernel_Name"]]
    step = None
    for s in reversed(starts):  # the last complete step
        if s + len(L) <= len(rows):
            step = rows[s:s + len(L)]
            break
    assert step is not None, "no complete step in the trace"
    print(f"# ResNet-50 batch {a.batch}: per-layer floors (HBM {a.hbm} TB/s, MFMA {a.peak} PF/s)\n")
    print("| # | layer | kernel | us | GB | TB/s | TFLOP | PF/s | floor us | eff |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    tot_us = tot_floor = tot_b = tot_f = 0.0
    for i, ((name, frag, byts, flops), r) in enumerate(zip(L, step)):
        kn = r["Kernel_Name"].replace("void ", "").replace("kvedge::(anonymous namespace)::", "")
        assert frag in kn or frag == "conv" and "conv" in kn and "seam" not in kn, (i, name, kn[:60])
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        floor = max(byts / (a.hbm * 1e12), flops / (a.peak * 1e15)) * 1e6
        tot_us += us
        tot_floor += floor
        tot_b += byts
        tot_f += flops
        short = kn.split("(")[0].replace("conv_", "").replace("_kernel", "")[:34]
        print(f"| {i} | {name} | {short} | {us:.1f} | {byts / 1e9:.3f} | {byts / us / 1e6:.2f} | "
              f"{flops / 1e12:.3f} | {flops / us / 1e9:.3f} | {floor:.1f} | {floor / us:.2f} |")
    print(f"\n**Step: {tot_us:.0f} us measured, {tot_floor:.0f} us sum of per-layer floors "
          f"({tot_floor / tot_us:.2f}); {tot_b / 1e9:.1f} GB compulsory HBM traffic, "
          f"{tot_f / 1e12:.2f} TFLOP ({tot_f / tot_us / 1e9:.3f} PF/s average).**")


if __name__ == "__main__":
    main()
