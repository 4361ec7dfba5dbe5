#!/usr/bin/env python3
"""Per-kernel time of ONE ResNet-50/YOLOv8n step as the bench runs it (autotuned tiles,
hipGraph replay).  Run under `rocprofv3 --kernel-trace --output-format csv`; a marker
kernel (non-graph synth_kernel on a tiny tensor) separates setup/autotune noise from the
measured replays, and `--summarize <kernel_trace.csv>` prints the per-kernel table."""
import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import torch
    from kvedge_amd import ops
    from kvedge_amd.engine import InferenceEngine

    assert ops.load()
    if a.model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50 as M
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n as M
    model = M.build(seed=0, device="cuda")
    eng = InferenceEngine(model, a.batch, M.image_size, device="cuda",
                          streams=a.streams).prepare(warmup=2)
    for _ in range(3):
        eng.run()
    torch.cuda.synchronize()
    marker = torch.empty(1, 8, 8, 3, dtype=torch.uint8, device="cuda")
    ops.synth_frames(marker, 0, 0)  # -> "synth_kernel": start of the measured region
    torch.cuda.synchronize()
    for _ in range(a.reps):
        eng.run()
    torch.cuda.synchronize()


def summarize(path, reps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = max(i for i, r in enumerate(rows) if "synth_kernel" in r["Kernel_Name"]
              and "dev" not in r["Kernel_Name"])
    body = rows[idx + 1:]
    agg = collections.OrderedDict()
    for r in body:
        name = r["Kernel_Name"].replace("void ", "").replace(
            "kvedge::(anonymous namespace)::", "").split("(")[0]
        key = (name[:110], r.get("Grid_Size_X", r.get("Grid_Size", "")))
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg.setdefault(key, []).append(dur)
    total = sum(sum(v) for v in agg.values()) / reps
    span = (int(body[-1]["End_Timestamp"]) - int(body[0]["Start_Timestamp"])) / 1e3 / reps
    print(f"# per-step kernel time {total:.1f} us, wall span per step {span:.1f} us "
          f"({len(body) // reps} kernels/step)\n")
    print("| kernel | grid | calls/step | us/step | % |\n|---|---|---|---|---|")
    for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        t = sum(v) / reps
        print(f"| {name} | {grid} | {len(v) // reps} | {t:.1f} | {100 * t / total:.1f} |")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--streams", type=int, default=1,
                    help="batch slices on HIP streams (the bench uses engine.BENCH_STREAMS)")
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize, a.reps)
    else:
        run(a)
