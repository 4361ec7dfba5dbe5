#!/usr/bin/env python3
"""Per-GPU batch sweep of the headline ResNet-50 step (hipGraph), one process."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="32,64,128,192,256,384,512")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops
    from kvedge_amd.engine import InferenceEngine

    assert ops.load()
    if a.model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50 as M
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n as M
    model = M.build(seed=0, device="cuda")
    res = []
    for b in [int(x) for x in a.batches.split(",")]:
        eng = InferenceEngine(model, b, M.image_size, device="cuda").prepare(warmup=2)
        for _ in range(3):
            eng.run()
        dt = eng.run_timed(a.steps)
        r = {"model": a.model, "batch": b, "images_per_s": round(b * a.steps / dt, 1),
             "ms_per_step": round(dt / a.steps * 1e3, 3)}
        print(json.dumps(r), flush=True)
        res.append(r)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
