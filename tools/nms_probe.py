#!/usr/bin/env python3
"""NMS workload at the bench shape: candidates per image over a batch of synthetic
frames, and the standalone nms kernel time."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kvedge_amd import ops  # noqa: E402
from kvedge_amd.models.yolov8 import STRIDES, KvYoloV8n as M  # noqa: E402

assert ops.load()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
m = M.build(seed=0, device="cuda")
fr = torch.empty(B, 640, 640, 3, dtype=torch.uint8, device="cuda")
ops.synth_frames(fr, 0, 3)
feats = m.heads(m.preprocess(fr))
boxes, scores, cls = ops.yolo_decode(feats, STRIDES, m.nc)
torch.cuda.synchronize()
cand = (scores > m.conf).sum(1).float()
print("candidates per image: min %d median %d max %d" % (cand.min(), cand.median(), cand.max()))
for conf in (m.conf, 0.5, 0.9):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ops.nms(boxes, scores, cls, conf, m.iou, m.max_det)
    torch.cuda.synchronize()
    st.record()
    for _ in range(10):
        dets, cnt = ops.nms(boxes, scores, cls, conf, m.iou, m.max_det)
    en.record()
    torch.cuda.synchronize()
    print("conf %.2f: nms %.1f us, kept max %d" % (conf, st.elapsed_time(en) / 10 * 1e3, cnt.max()))
