#!/usr/bin/env python3
"""Time the fused YOLO b0+b1 kernel (csrc/kernels/yolo_stem2.hip) vs the unfused pair at
batch --batch, 640x640 frames; run under rocprofv3 --pmc for counters."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=192)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only-fused", action="store_true")
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops
    from kvedge_amd.models.yolov8 import KvYoloV8n

    assert ops.load()
    m = KvYoloV8n.build(seed=0, device="cuda", calibrate=False)
    fr = torch.randint(0, 256, (a.batch, 640, 640, 3), dtype=torch.uint8, device="cuda")
    b0, b1 = m.b0_frames, m.b1

    def fused():
        return ops.yolo_stem2(fr, b0.spec, b0.w, b0.b, b1.spec, b1.w, b1.b)

    def pair():
        return b1(ops.stem_from_frames(fr, b0.spec, b0.w, b0.b))

    arms = [("fused", fused)] + ([] if a.only_fused else [("pair", pair)])
    for name, fn in arms:
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(5e6))
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name}: {e0.elapsed_time(e1) * 1e3 / a.iters:.1f} us", flush=True)


if __name__ == "__main__":
    main()
