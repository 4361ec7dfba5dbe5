#!/usr/bin/env python3
"""One summary line of a bench.py JSON output: headline img/s and ms/step, edge p50 (ms) and
img/s per batch, YOLOv8n img/s.   python tools/bench_line.py out.txt"""
import json
import sys


def main(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    ex = d.get("extra", {})
    parts = [f"headline {d['value']:.0f} ({d['ms_per_step']:.3f} ms)"]
    for e in ex.get("edge", []):
        parts.append(f"b{e['batch']} {e['p50_ms']:.4f} ms {e['images_per_s']:.0f}/s")
    y = ex.get("yolov8n")
    if isinstance(y, dict) and "value" in y:
        parts.append(f"yolo {y['value']:.0f}")
    print(" | ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
