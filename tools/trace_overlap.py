#!/usr/bin/env python3
"""Step-level overlap summary of rocprofv3 kernel traces of bench.py runs (one stream vs S
streams): wall time per step, sum of kernel durations, union busy time (time with at least
one kernel running), queues used, and per-kernel time per step side by side.

Steps are delimited by the frame-synthesis kernel (one per step); the last 3 steps are used.

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ps1 -o t -- python3 bench.py --streams 1
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ps2 -o t -- python3 bench.py --streams 2
  python tools/trace_overlap.py gpurun_out/ps1/t_kernel_trace.csv gpurun_out/ps2/t_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def load(path):
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"])
            for r in csv.DictReader(open(path))]
    rows.sort()
    return rows


def short(n):
    n = re.sub(r"void kvedge::\(anonymous namespace\)::", "", n)
    return n.split("(KvConvParams")[0].split("(")[0][:60]


def summarize(path, nsteps=3):
    rows = load(path)
    syn = [i for i, r in enumerate(rows) if "synth" in r[2]]
    a, b = syn[-(nsteps + 1)], syn[-1]
    seg = rows[a:b]
    wall = (rows[b][0] - rows[a][0]) / nsteps / 1e3
    busy = sum(r[1] - r[0] for r in seg) / nsteps / 1e3
    iv = sorted((r[0], r[1]) for r in seg)
    union, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    per = collections.defaultdict(float)
    for r in seg:
        per[short(r[2])] += (r[1] - r[0]) / nsteps / 1e3
    return {"wall_us": wall, "kernel_sum_us": busy, "union_busy_us": union / nsteps / 1e3,
            "queues": sorted(set(r[3] for r in seg)), "per_kernel": per}


def main(paths):
    sums = [summarize(p) for p in paths]
    print("| trace | wall us/step | sum of kernel us | union busy us | queues |")
    print("|---|---|---|---|---|")
    for p, s in zip(paths, sums):
        print(f"| {p} | {s['wall_us']:.0f} | {s['kernel_sum_us']:.0f} | {s['union_busy_us']:.0f} | "
              f"{len(s['queues'])} |")
    keys = sorted(set().union(*[s["per_kernel"] for s in sums]),
                  key=lambda k: -max(s["per_kernel"].get(k, 0.0) for s in sums))
    print("\n| kernel | " + " | ".join(f"trace {i} us/step" for i in range(len(paths))) + " |")
    print("|---" * (len(paths) + 1) + "|")
    for k in keys:
        print(f"| {k} | " + " | ".join(f"{s['per_kernel'].get(k, 0.0):.0f}" for s in sums) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
