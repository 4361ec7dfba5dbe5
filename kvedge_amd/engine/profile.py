"""Per-op HIP-event profiler for one eager step (SURVEY.md §5.1 tracing).

``rocprofv3 --kernel-trace`` is the ground truth (tools/profile_forward.py); this is the
in-process, always-available view: every public op in :mod:`kvedge_amd.ops` is wrapped so
that each call records a start/stop HIP event pair on torch's current stream.  One eager
(non-graph) step is run under it and the per-call device times are returned in call order
with the op name and the output shape.  ``bench.py --profile out.json`` writes it.
"""
from __future__ import annotations

import contextlib
import functools
import json
from typing import Dict, List

import torch

from .. import ops

_OPS = ("conv2d", "conv_dual", "conv_dual2", "conv_tail", "conv_pair", "c2f16", "stem_pool",
        "stem_pool_frames", "stem12_pool_frames", "stem_from_frames", "yolo_stem2", "maxpool2d",
        "sppf_pool", "global_avgpool", "pooled_fc", "softmax_rows", "upsample2x", "yolo_decode",
        "nms", "synth_frames", "preprocess", "batchnorm_nhwc")


def _shape_of(out):
    if isinstance(out, torch.Tensor):
        return list(out.shape)
    if isinstance(out, (tuple, list)) and out and isinstance(out[0], torch.Tensor):
        return list(out[0].shape)
    return None


@contextlib.contextmanager
def op_events(records: List[Dict]):
    """Wrap every kvedge op with a HIP event pair; appends dicts to ``records``."""
    saved = {}
    depth = [0]

    def wrap(name, fn):
        @functools.wraps(fn)
        def inner(*a, **kw):
            if depth[0] > 0 or not torch.cuda.is_available():
                return fn(*a, **kw)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            depth[0] += 1
            try:
                s.record()
                out = fn(*a, **kw)
                e.record()
            finally:
                depth[0] -= 1
            records.append({"op": name, "start": s, "stop": e, "shape": _shape_of(out)})
            return out
        return inner

    for name in _OPS:
        if hasattr(ops, name):
            saved[name] = getattr(ops, name)
            setattr(ops, name, wrap(name, saved[name]))
    try:
        yield records
    finally:
        for name, fn in saved.items():
            setattr(ops, name, fn)


def profile_step(engine) -> Dict:
    """One eager step of ``engine`` (graph bypassed) with per-op device times."""
    recs: List[Dict] = []
    torch.cuda.synchronize()
    with op_events(recs):
        engine._step()
    torch.cuda.synchronize()
    rows = []
    for r in recs:
        rows.append({"op": r["op"], "shape": r["shape"],
                     "ms": round(r["start"].elapsed_time(r["stop"]), 4)})
    total = sum(r["ms"] for r in rows)
    by_op: Dict[str, float] = {}
    for r in rows:
        by_op[r["op"]] = by_op.get(r["op"], 0.0) + r["ms"]
    return {"total_ms": round(total, 4), "calls": rows,
            "by_op_ms": {k: round(v, 4) for k, v in sorted(by_op.items(), key=lambda kv: -kv[1])}}


def write_profile(engine, path: str) -> Dict:
    prof = profile_step(engine)
    with open(path, "w") as f:
        json.dump(prof, f, indent=1)
    return prof
