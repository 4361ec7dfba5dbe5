#!/usr/bin/env python3
"""Standalone timing of the frames-in stems (ResNet stem12 + pool at batch 640, fused YOLO
b0 + b1 at batch 192) and the batch-1 split-K layers, for A/B of kernel builds on one box:

  KVEDGE_LIB=_C_ab.so python tools/stem_ab.py     # the variant build (tools/ab_build.sh)
  python tools/stem_ab.py                          # this tree's build

HIP-event median over ``--iters`` launches, a spin kernel queued first so the host stays
ahead.  Prints one JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    import torch

    fn()
    torch.cuda.synchronize()
    torch.cuda._sleep(int(min(5e7, 60_000 * iters)))
    evs = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
    return round(ts[len(ts) // 2], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    import torch

    from kvedge_amd import ops
    from kvedge_amd.models.resnet import KvResNet50, init_resnet50
    from kvedge_amd.models.yolov8 import KvYoloV8n, init_yolov8n

    assert ops.load(), "native library not built"
    out = {"lib": os.path.basename(ops.library_path())}
    g = torch.Generator().manual_seed(0)
    kv = KvResNet50(init_resnet50(seed=0), "cuda")
    fr = torch.randint(0, 256, (640, 224, 224, 3), dtype=torch.uint8, generator=g).cuda()
    y = torch.empty(640, 56, 56, 64, dtype=torch.bfloat16, device="cuda")
    out["stem12_b640_us"] = timed(
        lambda: ops.stem12_pool_frames(fr, kv.stem12_w, kv.stem.b, out=y), a.iters)
    yo = KvYoloV8n(init_yolov8n(seed=0, calibrate=False), "cuda")
    fy = torch.randint(0, 256, (192, 640, 640, 3), dtype=torch.uint8, generator=g).cuda()
    b0, b1 = yo.b0_frames, yo.b1
    yy = torch.empty(192, 160, 160, 32, dtype=torch.bfloat16, device="cuda")
    out["yolo_stem2_b192_us"] = timed(
        lambda: ops.yolo_stem2(fy, b0.spec, b0.w, b0.b, b1.spec, b1.w, b1.b, out=yy), a.iters)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
