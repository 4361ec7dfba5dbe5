#!/usr/bin/env python3
"""Per-layer table of the BENCH GRAPH itself (not of an eager forward, not of a probe).

The engine is built exactly as ``bench.py`` builds it (model, per-GPU batch, stream slices,
autotuned tiles, one hipGraph per step) and the graph is replayed ``--reps`` times after a
marker kernel, under ``rocprofv3 --kernel-trace``.  The summary step then assigns every
kernel of the replays to (slice, layer):

- the layer list comes from one instrumented eager forward of the slice shape
  (``tools/op_roofline.costs_only``): one row per op call, in call order, with its
  compulsory HBM bytes, FLOPs and pinned tile; an op is one kernel, or two for a split-K
  tile (GEMM + finalize, summed into the op's row), which the summary checks;
- kernels are matched to slices by the stream-order constraint: a slice's next kernel is
  the next op of its list and cannot start before that slice's previous kernel ended.

Per layer it reports the mean in-graph kernel duration (co-resident with the other slice's
kernels, as the bench runs it) and the layer's share of the step's WALL time: every
instant of the step is split evenly over the kernels running at that instant, so the
shares add up to the GPU's busy time and a layer that overlaps well costs less than its
duration.  This is the acceptance table of round 5 ("Next round" 1a).

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gl -o gl -- \\
      python3 tools/graph_layers.py run --labels gpurun_out/gl_labels.json
  python3 tools/graph_layers.py summarize gpurun_out/gl/.../gl_kernel_trace.csv \\
      --labels gpurun_out/gl_labels.json > profiles/<tag>_graph_layers.md
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import torch
    from kvedge_amd import ops
    from kvedge_amd.engine import BENCH_BATCH, BENCH_STREAMS, InferenceEngine
    from tools.op_roofline import costs_only

    assert ops.load(), "kvedge: HIP extension not loaded"
    if a.model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50 as M
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n as M
    batch = a.batch or BENCH_BATCH[a.model]
    streams = a.streams or BENCH_STREAMS[a.model]
    model = M.build(seed=0, device="cuda", calibrate=True)
    eng = InferenceEngine(model, batch, M.image_size, device="cuda", streams=streams)
    eng.prepare(warmup=2, autotune=not a.no_autotune)
    per = batch // streams
    # the labelled eager pass: a separator kernel (bn_kernel: the deployed models fold every
    # BatchNorm, so the forward never launches one) before the pass and after every op, so
    # the summary counts each op's kernels from the trace instead of assuming them (a Cout
    # split launches two, a split-K tile GEMM + finalize)
    sx = torch.zeros(1, 1, 1, 8, dtype=torch.bfloat16, device="cuda")
    sy, s1, s0 = torch.empty_like(sx), torch.ones(8, device="cuda"), torch.zeros(8, device="cuda")
    sep = lambda: ops.batchnorm_nhwc(sx, s1, s0, out=sy)  # noqa: E731
    torch.cuda.synchronize()
    with torch.no_grad():
        sep()
        rows = costs_only(model, eng.frames[:per], ops, after=sep)
    torch.cuda.synchronize()
    # kernels per op: a split-K tile is its GEMM and its finalize launch
    nk = [2 if (t is not None and ops.is_splitk(t)) else 1 for _, _, _, t in rows]
    with open(a.labels, "w") as f:
        json.dump({"model": a.model, "batch": batch, "streams": streams,
                   "rows": [[n, b, fl, t] for n, b, fl, t in rows], "kernels": nk}, f)
    for _ in range(3):
        eng.run()
    torch.cuda.synchronize()
    marker = torch.empty(1, 8, 8, 3, dtype=torch.uint8, device="cuda")
    ops.synth_frames(marker, 0, 0)  # "synth_kernel" (not synth_dev): start of the replays
    torch.cuda.synchronize()
    for _ in range(a.reps):
        eng.run()
    torch.cuda.synchronize()
    print(f"graph_layers: {a.model} b{batch} x{streams} streams, {len(rows)} ops per slice, "
          f"{a.reps} replays traced", flush=True)


def _short(name):
    name = name.replace("void ", "").replace("kvedge::(anonymous namespace)::", "")
    return name.split("(")[0]


def assign(kernels, op_of, n_slices):
    """kernels: [(start, end, name)] of one step sorted by start; op_of: the op index of each
    kernel position of a slice's sequence -> [(slice, op)] or None.  Greedy with the
    stream-order constraint; ties go to the slice that is further behind."""
    n_pos = len(op_of)
    ptr = [0] * n_slices
    last_end = [-1] * n_slices
    sig = [None] * n_pos  # kernel name per position, learned from the first slice there
    out = []
    for st, en, nm in kernels:
        cands = []
        for s in range(n_slices):
            p = ptr[s]
            if p >= n_pos:
                continue
            if sig[p] is not None and sig[p] != nm:
                continue
            slack = st - last_end[s]
            cands.append((slack < -2000, p, s))  # 2 us of timestamp skew tolerated
        if not cands:
            return None
        _, p, s = min(cands)
        sig[p] = sig[p] or nm
        out.append((s, op_of[p]))
        ptr[s] += 1
        last_end[s] = en
    return out if all(p == n_pos for p in ptr) else None


def _is_model_kernel(nm):
    return not (nm.startswith(("at::", "__amd_rocclr")) or "synth_dev" in nm or
                "bump_kernel" in nm)


def op_kernel_counts(names, n_ops):
    """Kernels per op of the labelled eager pass: ``names`` = kernel names in launch order up
    to the replay marker; the pass is the last n_ops + 1 separators (bn_kernel) and the
    model kernels between them.  None if the trace has no such pass (older labels)."""
    # demangled ("...::bn_kernel") or not ("_ZN6kvedge12_GLOBAL__N_19bn_kernelE...")
    sep = [i for i, nm in enumerate(names) if re.search(r"(^|::|\d)bn_kernel", nm)]
    if len(sep) < n_ops + 1:
        return None
    sep = sep[-(n_ops + 1):]
    return [sum(1 for nm in names[a + 1:b] if _is_model_kernel(nm))
            for a, b in zip(sep, sep[1:])]


def summarize(path, labels, reps, hbm, peak, out=sys.stdout):
    lab = json.load(open(labels))
    rows, n_sl = lab["rows"], lab["streams"]
    n_ops = len(rows)
    recs = list(csv.DictReader(open(path)))
    recs.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = max(i for i, r in enumerate(recs) if "synth_kernel" in r["Kernel_Name"]
              and "synth_dev" not in r["Kernel_Name"])
    nk = op_kernel_counts([_short(r["Kernel_Name"]) for r in recs[:idx]], n_ops)
    if nk is None:
        nk = lab.get("kernels") or [1] * n_ops
    op_of = [p for p in range(n_ops) for _ in range(nk[p])]
    body = recs[idx + 1:]
    # steps start at the frame kernel (synth_dev_kernel) of each replay
    starts = [i for i, r in enumerate(body) if "synth_dev_kernel" in r["Kernel_Name"]]
    if len(starts) < reps:
        raise SystemExit(f"found {len(starts)} replays, expected {reps}")
    dur = collections.defaultdict(list)       # op -> [us]
    share = collections.defaultdict(float)    # op -> wall-share us (summed over steps)
    names = {}
    walls, busy = [], []
    extra_share = collections.defaultdict(float)
    for k, s0 in enumerate(starts):
        s1 = starts[k + 1] if k + 1 < len(starts) else len(body)
        step = body[s0:s1]
        t0 = int(step[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in step)
        walls.append((t1 - t0) / 1e3)
        ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"]))
              for r in step]
        model_ks = [x for x in ks if _is_model_kernel(x[2])]
        other = [x for x in ks if x not in model_ks]
        if len(model_ks) != len(op_of) * n_sl:
            if k == 0 and len(model_ks) % n_sl == 0:
                # an op launched an unexpected number of kernels: fall back to one row per
                # kernel position of the slice sequence (labels are then kernel names)
                import collections as _c
                print(f"# note: {len(model_ks)} kernels per step for {len(op_of)} op kernels x "
                      f"{n_sl} slices; rows are kernel positions, not ops: "
                      f"{dict(_c.Counter(x[2][:40] for x in model_ks))}", file=sys.stderr)
                n_ops = len(model_ks) // n_sl
                op_of = list(range(n_ops))
                nk = [1] * n_ops
                rows = [[f"kernel #{i}", 0, 0.0, None] for i in range(n_ops)]
            else:
                raise SystemExit(f"step {k}: {len(model_ks)} model kernels, expected "
                                 f"{len(op_of)} (of {n_ops} ops) x {n_sl} slices")
        asg = assign(model_ks, op_of, n_sl)
        if asg is None:
            raise SystemExit(f"step {k}: kernels do not match the op order of any slice")
        lab_of = {}
        for (st, en, nm), (s, p) in zip(model_ks, asg):
            dur[p].append((en - st) / 1e3)
            names[p] = names.get(p) or nm  # an op's first kernel names it
            lab_of[(st, en, nm)] = p
        # wall share: sweep the union of intervals, split each segment over active kernels
        ev = []
        for x in ks:
            ev.append((x[0], 1, x))
            ev.append((x[1], -1, x))
        ev.sort(key=lambda e: (e[0], -e[1]))
        active, prev, b = [], None, 0.0
        for t, kind, x in ev:
            if prev is not None and active and t > prev:
                seg = (t - prev) / 1e3
                b += seg
                for y in active:
                    if y in lab_of:
                        share[lab_of[y]] += seg / len(active)
                    else:
                        extra_share[y[2]] += seg / len(active)
            if kind == 1:
                active.append(x)
            else:
                active.remove(x)
            prev = t
        busy.append(b)
    nst = len(starts)
    wall = sorted(walls)[len(walls) // 2]
    print(f"# {lab['model']} bench graph, batch {lab['batch']} as {n_sl} slice(s) of "
          f"{lab['batch'] // n_sl}: per-layer in-graph times ({nst} replays, rocprofv3 "
          f"kernel trace)\n", file=out)
    print(f"Step wall (first kernel start -> last kernel end, median): **{wall:.1f} us**; "
          f"GPU busy (union of kernel intervals) {sum(busy) / nst:.1f} us; "
          f"{n_ops} ops per slice.\n", file=out)
    print("`dur` = mean kernel duration in the graph (co-resident with the other slice); "
          "`wall share` = the layer's share of the step's busy time, summed over slices "
          "(each instant split evenly over the kernels running then); floors per slice at "
          f"HBM {hbm} TB/s / MFMA {peak} PF/s.\n", file=out)
    print("| # | op | tile | kernel | dur us | floor us | eff | wall share us | % step |",
          file=out)
    print("|---|---|---|---|---|---|---|---|---|", file=out)
    from tools.op_roofline import family

    tot_share = 0.0
    for p in range(n_ops):
        nm, byts, flops, tile = rows[p]
        d = sum(dur[p]) / (nst * n_sl)  # an op's kernels summed, per slice and step
        fl = max(byts / (hbm * 1e12), flops / (peak * 1e15)) * 1e6
        sh = share[p] / nst
        tot_share += sh
        kname = names[p][:60] + (f" (+{nk[p] - 1} kernel{'s' if nk[p] > 2 else ''})"
                                 if nk[p] > 1 else "")
        print(f"| {p} | {nm} | {family(tile)} | {kname} | {d:.1f} | {fl:.1f} | "
              f"{fl / max(d, 1e-3):.2f} | {sh:.1f} | {100 * sh / wall:.1f} |", file=out)
    oth = sum(extra_share.values()) / nst
    print(f"\nModel layers: {tot_share:.1f} us of wall share; frames/concat/other kernels: "
          f"{oth:.1f} us.\n", file=out)
    worst = sorted(range(n_ops), key=lambda p: -share[p])[:10]
    print("Largest wall shares: " + ", ".join(f"#{p} {rows[p][0]} ({share[p] / nst:.0f} us)"
                                             for p in worst), file=out)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--model", default="resnet50", choices=["resnet50", "yolov8n"])
    r.add_argument("--batch", type=int, default=0, help="0 = engine.BENCH_BATCH")
    r.add_argument("--streams", type=int, default=0, help="0 = engine.BENCH_STREAMS")
    r.add_argument("--reps", type=int, default=5)
    r.add_argument("--no-autotune", action="store_true")
    r.add_argument("--labels", required=True)
    s = sub.add_parser("summarize")
    s.add_argument("trace", help="kernel_trace.csv, or a directory to search")
    s.add_argument("--labels", required=True)
    s.add_argument("--reps", type=int, default=5)
    s.add_argument("--hbm", type=float, default=6.0)
    s.add_argument("--peak", type=float, default=2.5)
    a = ap.parse_args()
    if a.cmd == "run":
        run(a)
    else:
        path = a.trace
        if os.path.isdir(path):
            path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"),
                                    recursive=True))[-1]
        summarize(path, a.labels, a.reps, a.hbm, a.peak)


if __name__ == "__main__":
    main()
