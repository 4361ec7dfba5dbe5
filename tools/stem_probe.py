#!/usr/bin/env python3
"""Time the fused stem+maxpool kernel (csrc/kernels/stem_pool.hip) at a given batch.
Variant knob: KVEDGE_STEM_THREADS=256|512 (read once per process)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops
    from kvedge_amd.models.resnet import KvResNet50

    assert ops.load()
    m = KvResNet50.build(seed=0, device="cuda", calibrate=False)
    fr = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device="cuda")
    x = m.preprocess(fr)
    flops = 2 * a.batch * 112 * 112 * 64 * 147
    def frames16():
        m.stem12 = False
        return m.stem_and_pool(fr, frames_in=True)

    def frames12():
        m.stem12 = True
        return m.stem_and_pool(fr, frames_in=True)

    for name, fn in (("preprocess+stem_pool", lambda: m.stem_and_pool(m.preprocess(fr))),
                     ("stem_pool", lambda: m.stem_and_pool(x)),
                     ("stem_pool_frames (16-ch s2d, K 256)", frames16),
                     ("stem12_pool_frames (12-ch s2d, K 192)", frames12)):
        out = fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.reps * 1e3
        print(f"{name} threads={os.environ.get('KVEDGE_STEM_THREADS', 'default')} "
              f"batch={a.batch}: {us:.1f} us  ({flops / us / 1e6:.0f} TF/s model-FLOP)  "
              f"checksum={float(out.float().sum()):.6g}")


if __name__ == "__main__":
    main()
