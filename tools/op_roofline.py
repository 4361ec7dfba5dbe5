#!/usr/bin/env python3
"""Per-layer roofline of one forward, measured per op call (no trace matching).

Every kernel-launching entry point of ``kvedge_amd.ops`` the model calls is wrapped for one
eager forward: a HIP event pair brackets the call, and the wrapper derives the launch's
compulsory HBM bytes (operands read once, outputs written once, strided 1x1 sources counted
at the pixels they read) and its model FLOPs (2 x MACs of the real convolution; stems at
their real taps, not the s2d-padded K) from the call's own arguments.  A spin kernel queued
first keeps the host ahead of the GPU, so each event pair spans the op's kernels only, not
host launch gaps.  Tiles are the autotuner's (the engine is prepared as bench.py prepares
it, at ``--batch x --streams``, so the per-slice shapes are the bench's).

Floors: HBM at --hbm TB/s, MFMA at --peak PF/s; 'floor' is the larger, 'eff' =
floor / measured.  Works for both models (the ResNet-50 trace-matched table is
tools/roofline_table.py; this one needs no layer list, which is what YOLOv8n lacked).

  python tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > yolo_roofline.md
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# kernel-family boundaries of kv_conv2d's tile index (csrc/kernels/conv_igemm.hip)
FAMILIES = [(0, "v1"), (6, "glds"), (32, "stream"), (54, "direct"), (58, "nloop"),
            (68, "xp/bk32/de"), (86, "splitk"), (105, "direct-de"),
            (108, "skinny"), (117, "pp")]  # pp 117: 256x256, 118: 512x128, 119-120: persistent


def family(tile):
    if tile is None or tile < 0:
        return "heur"
    name = FAMILIES[0][1]
    for lo, n in FAMILIES:
        if tile >= lo:
            name = n
    return f"{name}:{tile}"


def _b(t, c=None):
    """bf16/any tensor bytes, or of its first c channels (NHWC slice)."""
    if c is None:
        return t.numel() * t.element_size()
    return t.numel() // t.shape[-1] * c * t.element_size()


def conv2d_cost(x, spec, w, bias, res=None, out=None, x_coff=0, y_coff=0, r_coff=0, tile=-1):
    N, H, W, _ = x.shape
    Ho, Wo = spec.out_hw(H, W)
    m = N * Ho * Wo
    stem = spec.cin == 16 and spec.pad_b >= 0
    if spec.kh == 1 and spec.stride > 1:
        rd = m * spec.cin * 2
    else:
        rd = N * H * W * spec.cin * 2
    wr = m * spec.cout * 2 * (2 if res is not None else 1)
    k = 27 if stem else spec.kh * spec.kw * spec.cin
    if stem:
        name = f"stem 3x3/2 3>{spec.cout} as s2d {spec.kh}x{spec.kw} @{H}x{W}"
    else:
        name = (f"conv {spec.kh}x{spec.kw}/{spec.stride} {spec.cin}>{spec.cout} @{H}x{W}"
                + (" +res" if res is not None else ""))
    return name, rd + wr + _b(w), 2.0 * m * k * spec.cout, tile


def conv_dual_cost(x1, x2, w, bias, act, stride2, out=None, tile=-1):
    N, Ho, Wo, K1 = x1.shape
    K2, co = x2.shape[3], w.shape[0]
    m = N * Ho * Wo
    return (f"dual 1x1 {K1}+{K2}>{co} @{Ho}x{Wo}" + (" s2" if stride2 > 1 else ""),
            (m * (K1 + K2) + m * co) * 2 + _b(w),
            2.0 * m * (K1 + K2) * co, tile)


def conv_dual2_cost(x, K1, x2, w, bias, act, out, x_coff=0, x2_coff=0, y_coff=0, stride2=1,
                    up2=False, tile=-1):
    N, Ho, Wo, _ = x.shape
    co = w.shape[0]
    K2 = w.shape[1] - K1
    m = N * Ho * Wo
    # x2 is read at its own resolution: the up2 form reads each half-resolution pixel once
    m2 = m // 4 if up2 else m
    tag = " up2" if up2 else (" s2" if stride2 > 1 else "")
    return (f"dual 1x1 {K1}+{K2}>{co} @{Ho}x{Wo}{tag}", (m * K1 + m2 * K2 + m * co) * 2 + _b(w),
            2.0 * m * (K1 + K2) * co, tile)


def conv_tail_cost(x, w, bias, act, w1, b1, res=None, x2=None, stride2=1, out=None, z=None,
                   tile=-1):
    N, H, W, K1 = x.shape
    m = N * H * W
    co, nt = w.shape[0], w1.shape[0]
    k = w.shape[1]
    rd = m * K1 * 2 + (m * (k - K1) * 2 if x2 is not None else m * co * 2)
    return (f"tail {k}>{co}>{nt} @{H}x{W}", rd + m * (co + nt) * 2,
            2.0 * m * (k * co + co * nt), tile)


def conv_pair_cost(x, spec, w, bias, w2, b2, out, x_coff=0, z_coff=0, tile=0):
    N, H, W, _ = x.shape
    m = N * H * W
    c2 = w2.shape[0]
    return (f"pair 3x3 {spec.cin}>{spec.cout} + 1x1 >{c2} @{H}x{W} (direct {tile})",
            m * (spec.cin + c2) * 2 + _b(w) + _b(w2),
            2.0 * m * (9 * spec.cin * spec.cout + spec.cout * c2), None)


def stem_from_frames_cost(frames, spec, w, bias, out=None, tile=-1):
    N, H, W, _ = frames.shape
    m = N * (H // 2) * (W // 2)
    return (f"stem 3x3/2 3>{spec.cout} (frames in) @{H}x{W}", frames.numel() + m * spec.cout * 2,
            2.0 * m * 27 * spec.cout, tile)


def stem12_cost(frames, w12, bias, out=None, y_coff=0, mean=None, std=None):
    N, H, W, _ = frames.shape
    m = N * (H // 2) * (W // 2)
    return ("stem 7x7/2 3>64 + pool (frames in)", frames.numel() + N * (H // 4) * (W // 4) * 128,
            2.0 * m * 147 * 64, None)


def yolo_stem2_cost(frames, spec0, w0, b0, spec1, w1, b1, out=None):
    N, H, W, _ = frames.shape
    m0, m1 = N * (H // 2) * (W // 2), N * (H // 4) * (W // 4)
    return ("stem 3x3/2 3>16 + b1 3x3/2 16>32 (frames in, fused)", frames.numel() + m1 * 64,
            2.0 * (m0 * 27 * 16 + m1 * 144 * 32), None)


def c2f16_cost(x, w1, b1, wm1, bm1, wm2, bm2, w2, b2, out=None, x_coff=0, y_coff=0, S=0):
    N, H, W, _ = x.shape
    m = N * H * W
    wb = _b(w1) + _b(wm1) + _b(wm2) + _b(w2)
    # x (32 channels) read once, y (32) written once; MACs 32*32 + 2*144*16 + 48*32 per pixel
    return (f"c2f fused 32>[16|16+3x3x2]>32 @{H}x{W}", m * 64 * 2 + wb,
            2.0 * m * (1024 + 2 * 2304 + 1536), None)


def sppf_cost(buf, C):
    return f"sppf pools c{C}", _b(buf, C) * 4, 0.0, None


def upsample_cost(x, out, C=None, x_coff=0, y_coff=0):
    C = C or (x.shape[3] - x_coff)
    return f"upsample2x c{C} @{x.shape[1]}", _b(x, C) * 5, 0.0, None


def decode_cost(feats, strides, nc, boxes=None, scores=None, cls=None):
    rd = sum(_b(f) for f in feats)
    a = sum(f.shape[1] * f.shape[2] for f in feats) * feats[0].shape[0]
    return "yolo decode", rd + a * 6 * 4, 0.0, None


def nms_cost(boxes, scores, cls, conf=0.25, iou=0.7, max_det=300, out=None, count=None):
    return "nms", _b(boxes) + _b(scores) + _b(cls) + scores.shape[0] * max_det * 24, 0.0, None


def avgpool_cost(x, out=None):
    return "global avgpool", _b(x) + x.shape[0] * x.shape[3] * 2, 0.0, None


def softmax_cost(x, out=None, argmax=None):
    return "softmax + top1", _b(x) + x.numel() * 4, 0.0, None


COSTS = {"conv2d": conv2d_cost, "conv_dual": conv_dual_cost, "conv_dual2": conv_dual2_cost,
         "conv_tail": conv_tail_cost,
         "conv_pair": conv_pair_cost, "c2f16": c2f16_cost,
         "stem_from_frames": stem_from_frames_cost, "stem12_pool_frames": stem12_cost,
         "yolo_stem2": yolo_stem2_cost,
         "sppf_pool": sppf_cost, "upsample2x": upsample_cost, "yolo_decode": decode_cost,
         "nms": nms_cost, "global_avgpool": avgpool_cost, "softmax_rows": softmax_cost}


def costs_only(model, frames, ops, after=None):
    """The op rows of one forward without timing (CPU works): [(name, bytes, flops, tile)].
    ``after``: called after every recorded (outermost) op -- tools/graph_layers.py launches a
    separator kernel there, so the trace shows how many kernels each op launched."""
    recs, saved = [], {}
    for fname, cost in COSTS.items():
        saved[fname] = fn = getattr(ops, fname)

        def w(*args, _fn=fn, _cost=cost, **kw):
            # an op that falls back to other wrapped ops (a tail whose seam the kernel
            # refuses runs two conv2d) is recorded as those ops: one row per launch
            row, n0 = _cost(*args, **kw), len(recs)
            r = _fn(*args, **kw)
            if len(recs) == n0:
                recs.append(row)
                if after is not None:
                    after()
            return r
        setattr(ops, fname, w)
    try:
        model(frames)
    finally:
        for fname, fn in saved.items():
            setattr(ops, fname, fn)
    return recs


def measure(model, frames, torch, ops):
    """One eager forward with every op in COSTS bracketed by events -> rows."""
    recs = []
    saved = {}

    def wrap(fname, fn, cost):
        def w(*args, **kw):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            n0 = len(recs)
            e0.record()
            r = fn(*args, **kw)
            e1.record()
            if len(recs) == n0:  # nested wrapped ops already timed themselves
                recs.append((cost(*args, **kw), e0, e1))
            return r
        return w

    for fname, cost in COSTS.items():
        saved[fname] = getattr(ops, fname)
        setattr(ops, fname, wrap(fname, saved[fname], cost))
    try:
        torch.cuda._sleep(int(2e8))  # host runs ahead: events time kernels, not launches
        with torch.no_grad():
            model(frames)
        torch.cuda.synchronize()
    finally:
        for fname, fn in saved.items():
            setattr(ops, fname, fn)
    return [(c, e0.elapsed_time(e1) * 1e3) for c, e0, e1 in recs]


def table(rows, title, hbm, peak, out=sys.stdout):
    print(f"# {title}: per-op floors (HBM {hbm} TB/s, MFMA {peak} PF/s)\n", file=out)
    print("| # | op | tile | us | GB | TB/s | TFLOP | PF/s | floor us | eff | lost us |", file=out)
    print("|---|---|---|---|---|---|---|---|---|---|---|", file=out)
    tot = dict(us=0.0, floor=0.0, b=0.0, f=0.0)
    for i, ((name, byts, flops, tile), us) in enumerate(rows):
        floor = max(byts / (hbm * 1e12), flops / (peak * 1e15)) * 1e6
        tot["us"] += us
        tot["floor"] += floor
        tot["b"] += byts
        tot["f"] += flops
        print(f"| {i} | {name} | {family(tile)} | {us:.1f} | {byts / 1e9:.3f} | "
              f"{byts / max(us, 1e-3) / 1e6:.2f} | {flops / 1e12:.3f} | "
              f"{flops / max(us, 1e-3) / 1e9:.3f} | {floor:.1f} | {floor / max(us, 1e-3):.2f} | "
              f"{us - floor:.1f} |", file=out)
    print(f"\n**Forward: {tot['us']:.0f} us measured, {tot['floor']:.0f} us sum of per-op floors "
          f"({tot['floor'] / max(tot['us'], 1e-3):.2f}); {tot['b'] / 1e9:.2f} GB compulsory HBM "
          f"traffic, {tot['f'] / 1e12:.2f} TFLOP ({tot['f'] / max(tot['us'], 1e-3) / 1e9:.3f} "
          f"PF/s average).**\n", file=out)
    worst = sorted(range(len(rows)), key=lambda i: -(rows[i][1] - max(
        rows[i][0][1] / (hbm * 1e12), rows[i][0][2] / (peak * 1e15)) * 1e6))[:8]
    print("Largest gaps (us above floor): " + ", ".join(
        f"#{i} {rows[i][0][0]}" for i in worst), file=out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="yolov8n", choices=["resnet50", "yolov8n"])
    ap.add_argument("--batch", type=int, default=192, help="per-slice batch")
    ap.add_argument("--streams", type=int, default=2, help="engine slices (autotune context)")
    ap.add_argument("--hbm", type=float, default=6.0)
    ap.add_argument("--peak", type=float, default=2.5)
    ap.add_argument("--reps", type=int, default=3, help="median over this many forwards")
    a = ap.parse_args()

    import torch
    from kvedge_amd import ops
    from kvedge_amd.engine import InferenceEngine

    assert ops.load(), "kvedge: HIP extension not loaded"
    if a.model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50 as M
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n as M
    model = M.build(seed=0, device="cuda")
    eng = InferenceEngine(model, a.batch * a.streams, M.image_size, device="cuda",
                          streams=a.streams).prepare(warmup=2)
    eng.run()
    torch.cuda.synchronize()
    frames = eng.frames[:a.batch].clone()
    runs = [measure(model, frames, torch, ops) for _ in range(a.reps + 1)][1:]
    rows = [(runs[0][i][0], sorted(r[i][1] for r in runs)[len(runs) // 2])
            for i in range(len(runs[0]))]
    table(rows, f"{a.model} batch {a.batch} (one slice of {a.batch * a.streams}, eager, "
                f"autotuned tiles)", a.hbm, a.peak)


if __name__ == "__main__":
    main()
