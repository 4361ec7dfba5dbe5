#!/usr/bin/env python3
"""Sweep of the headline ResNet-50 step (hipGraph, autotuned tiles) over per-GPU batch
and early-stage micro-batching, one process.

  --configs "256:0:0,256:64:3"   batch:microbatch:microbatch_blocks
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="64:0:0,128:0:0,256:0:0,512:0:0,256:64:3,256:32:3,"
                                          "256:64:7,256:32:7,512:64:3,512:64:7")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--out", default="gpurun_out/sweep.jsonl")
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
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    for cfg in a.configs.split(","):
        b, mb, nb = (int(v) for v in cfg.split(":"))
        if hasattr(model, "microbatch"):
            model.microbatch, model.microbatch_blocks = mb, nb
        eng = InferenceEngine(model, b, M.image_size, device="cuda").prepare(warmup=2)
        for _ in range(3):
            eng.run()
        dt = eng.run_timed(a.steps)
        lat = eng.measure_latency(a.steps)  # synchronised per step: edge-module latency
        r = {"model": a.model, "batch": b, "microbatch": mb, "mb_blocks": nb,
             "images_per_s": round(b * a.steps / dt, 1), "ms_per_step": round(dt / a.steps * 1e3, 3),
             "latency_p50_ms": round(lat.percentile(50), 3),
             "latency_p99_ms": round(lat.percentile(99), 3)}
        print(json.dumps(r), flush=True)
        with open(a.out, "a") as f:
            f.write(json.dumps(r) + "\n")
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
