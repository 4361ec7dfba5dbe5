#!/usr/bin/env python3
"""How many YOLO anchors pass the confidence threshold with the seeded random-init
weights (sizes the NMS work: candidates to sort and suppress per image)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kvedge_amd import ops  # noqa: E402
from kvedge_amd.models.yolov8 import STRIDES, KvYoloV8n as M  # noqa: E402

assert ops.load()
m = M.build(seed=0, device="cuda")
fr = torch.empty(8, 640, 640, 3, dtype=torch.uint8, device="cuda")
ops.synth_frames(fr, 0, 0)
feats = m.heads(m.preprocess(fr))
boxes, scores, cls = ops.yolo_decode(feats, STRIDES, m.nc)
dets, cnt = ops.nms(boxes, scores, cls, m.conf, m.iou, m.max_det)
torch.cuda.synchronize()
print("candidates > conf per image:", (scores > m.conf).sum(1).tolist())
print("kept per image:", cnt.tolist())
print("score quantiles:", torch.quantile(scores[0].float(), torch.tensor([0.5, 0.9, 0.99], device="cuda")).tolist())
