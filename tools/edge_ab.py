#!/usr/bin/env python3
"""Same-box A/B of the edge operating points (bench.py ``extra.edge``) over the tile table.

An arm is a set of knobs (``KEY=VAL,KEY=VAL``; arms separated by ``;``): environment variables
read when the engine is built and tuned (``KVEDGE_TILE_LIMIT``: the tuner sees the first N
tiles only, 0 = the whole table), ``KVEDGE_TAIL1_MIN_ROWS`` (models.resnet.TAIL1_MIN_ROWS,
the stage-1 fused-tail gate) and ``KVEDGE_SEAM_MIN_WGS`` (ops.SEAM_MIN_WGS, the v9 seam gate).  Per arm the engine of every batch is rebuilt and autotuned,
then ``--steps`` synchronised replays give p50 / p99.  Arms alternate ``--rounds`` times so box drift hits both alike.  Prints one
JSON line per (round, arm, batch) and a summary of the median p50 per arm.

  python tools/edge_ab.py --arms "KVEDGE_TILE_LIMIT=108;KVEDGE_TILE_LIMIT=0" --rounds 2
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="KVEDGE_TILE_LIMIT=108;KVEDGE_TILE_LIMIT=0")
    ap.add_argument("--batches", default="1,8,64")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops
    from kvedge_amd.engine import edge_latency
    from kvedge_amd.models import resnet
    from kvedge_amd.models.resnet import KvResNet50

    assert ops.load(), "kvedge: HIP extension not loaded"
    model = KvResNet50.build(seed=0, device="cuda", calibrate=True)
    batches = [int(b) for b in a.batches.split(",")]
    arms = [dict(kv.split("=", 1) for kv in arm.split(",") if kv) for arm in a.arms.split(";")]
    keys = sorted({k for arm in arms for k in arm})
    base = {k: os.environ.get(k) for k in keys}
    tail0 = resnet.TAIL1_MIN_ROWS
    seam0 = ops.SEAM_MIN_WGS
    res = {}
    for r in range(a.rounds):
        for arm in arms:
            for k in keys:  # unset knobs fall back to the process's own value
                v = arm.get(k, base[k])
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            resnet.TAIL1_MIN_ROWS = int(os.environ.get("KVEDGE_TAIL1_MIN_ROWS", tail0))
            ops.SEAM_MIN_WGS = int(os.environ.get("KVEDGE_SEAM_MIN_WGS", seam0))
            tag = ",".join(f"{k}={v}" for k, v in sorted(arm.items()))
            for row in edge_latency(model, KvResNet50.image_size, batches, steps=a.steps):
                row.update(round=r, arm=tag)
                print(json.dumps(row), flush=True)
                res.setdefault((tag, row["batch"]), []).append(row["p50_ms"])
    torch.cuda.synchronize()
    for (tag, b), v in sorted(res.items()):
        print(json.dumps({"summary": True, "arm": tag, "batch": b,
                          "p50_ms_median": round(statistics.median(v), 4), "p50_ms": v}))


if __name__ == "__main__":
    main()
