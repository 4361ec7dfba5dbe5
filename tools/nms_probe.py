#!/usr/bin/env python3
"""Time the YOLOv8n NMS kernel on the model's own decode output (random-init weights, synthetic
frames), with KVEDGE_NMS_DIAG switching phases off (timing only; 1 = no greedy suppression,
2 = no top-set sort) -- where the per-image NMS latency goes.

  python tools/nms_probe.py --batch 192
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=192)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    from kvedge_amd import ops
    from kvedge_amd.models.yolov8 import STRIDES, KvYoloV8n

    assert ops.load()
    m = KvYoloV8n.build(seed=0, device="cuda")
    fr = torch.randint(0, 256, (a.batch, 640, 640, 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(1)).cuda()
    with torch.no_grad():
        feats = m.heads(m.stem_b1(fr), b1_done=True)
        boxes, scores, cls = ops.yolo_decode(feats, STRIDES, m.nc)
    torch.cuda.synchronize()
    print(f"candidates per image > conf {m.conf}: "
          f"{float((scores > m.conf).sum(1).float().mean()):.0f} of {scores.shape[1]}")
    os.environ["KVEDGE_NMS_DIAG"] = "4"
    out, cnt = ops.nms(boxes, scores, cls, m.conf, m.iou, m.max_det)
    torch.cuda.synchronize()
    ph = out[:, 0, :3].float().cpu() / 100.0  # 10-ns ticks -> us
    print("per-image phase us (median over images): compaction+select %.1f, sort %.1f, "
          "suppression %.1f" % tuple(float(ph[:, i].median()) for i in range(3)))
    print("per-image phase us (max over images):    compaction+select %.1f, sort %.1f, "
          "suppression %.1f" % tuple(float(ph[:, i].max()) for i in range(3)))
    nc = (scores > m.conf).sum(1)
    print(f"candidates per image: max {int(nc.max())}, images over 1024: {int((nc > 1024).sum())}")
    for d in ("0", "8", "1", "2", "3"):  # 8: the bucket top-set sort instead of the bitonic
        os.environ["KVEDGE_NMS_DIAG"] = d
        ts = []
        for _ in range(a.iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out, cnt = ops.nms(boxes, scores, cls, m.conf, m.iou, m.max_det)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        ts.sort()
        extra = f" kept/image {float(cnt.float().mean()):.0f}" if d == "0" else ""
        print(f"diag {d}: {ts[len(ts) // 2]:.1f} us{extra}", flush=True)
    os.environ.pop("KVEDGE_NMS_DIAG")


if __name__ == "__main__":
    main()
