"""Print the autotuner's per-layer picks (tile, us) for the bench configuration.
  python tools/tune_report.py [--model resnet50] [--streams 2] [--batch 1280]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--streams", type=int, default=0)
    ap.add_argument("--batch", type=int, default=0)
    a = ap.parse_args()
    from kvedge_amd import ops
    from kvedge_amd.engine import BENCH_BATCH, BENCH_STREAMS, InferenceEngine

    assert ops.load()
    B = a.batch or BENCH_BATCH[a.model]
    S = a.streams or BENCH_STREAMS[a.model]
    if a.model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50 as M
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n as M
    model = M.build(seed=0, device="cuda")
    eng = InferenceEngine(model, B, M.image_size, device="cuda", streams=S)
    eng.prepare(warmup=1)
    for k, (tile, us) in eng.tuning.items():
        print(f"{tile:3d} {us!s:>9} us  {k}")


if __name__ == "__main__":
    main()
