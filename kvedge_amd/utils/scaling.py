"""Data-parallel scaling curve of the headline bench ("images/sec at 1/2/4/8
GPUs with scaling curve JSON").

The reference has no benchmark at all; BASELINE.json names the metric
"images/sec ResNet-50 edge module at 1/2/4/8 MI355X".  This runner starts ``bench.py --gpus N``
once per N as a child process (each self-launches N ranks, one per GPU over RCCL), collects
each run's one JSON line, and writes the curve:

  {"metric": ..., "model": ..., "points": [{"n_gpus": N, "value": img/s, "per_gpu": ...,
   "ms_per_step": ..., "efficiency": per_gpu(N) / per_gpu(N0)}, ...], "base_n": N0}

Weak scaling: per-GPU batch is fixed, so ideal efficiency is 1.0 at every N.  The parent never
touches the GPU (it counts devices from the KFD topology in sysfs, never through HIP), so
the children start on clean devices.

  python -m kvedge_amd.utils.scaling --gpus 1,2,4,8 --out gpurun_out/scaling.json
  python -m kvedge_amd.utils.scaling --cpu --gpus 1,2 --steps 1 --warmup 0   # gloo rehearsal
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_point(n: int, bench_args: List[str], timeout: float = 1800.0) -> Dict:
    """One ``bench.py --gpus n`` child; returns its JSON line (raises on failure)."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)  # the child self-launches its own ranks
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)] + bench_args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    if r.returncode != 0 or not lines:
        raise RuntimeError(f"bench.py --gpus {n} failed (rc {r.returncode}):\n"
                           f"{r.stdout[-2000:]}\n{r.stderr[-4000:]}")
    return json.loads(lines[-1])


def curve(results: List[Dict]) -> Dict:
    """Scaling curve from bench JSON lines (any order); efficiency vs the smallest N."""
    pts = sorted(results, key=lambda d: d["n_gpus"])
    base = pts[0]
    base_per = base["value"] / base["n_gpus"]
    out = []
    for d in pts:
        per = d["value"] / d["n_gpus"]
        out.append({"n_gpus": d["n_gpus"], "value": d["value"], "per_gpu": round(per, 2),
                    "ms_per_step": d["ms_per_step"],
                    "efficiency": round(per / base_per, 4) if base_per > 0 else None,
                    "replica_ok": d.get("extra", {}).get("replica_check", {}).get("ok")})
    return {"metric": base["metric"], "unit": base.get("unit"), "scaling": base.get("scaling"),
            "model": base["config"]["model"], "per_gpu_batch": base["config"].get("per_gpu_batch"),
            "dtype": base.get("dtype"), "data": base.get("data"), "base_n": base["n_gpus"],
            "points": out}


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", default="1,2,4,8", help="comma-separated GPU counts")
    ap.add_argument("--out", default="", help="write the curve JSON here")
    ap.add_argument("--cpu", action="store_true", help="gloo rehearsal on the CPU")
    ap.add_argument("--timeout", type=float, default=1800.0, help="per point, seconds")
    a, rest = ap.parse_known_args(argv)  # everything else goes to bench.py
    ns = [int(x) for x in a.gpus.split(",") if x]
    if not a.cpu:
        from kvedge_amd.parallel import visible_gpu_count

        ndev = visible_gpu_count()  # sysfs: this parent never initialises HIP
        skipped = [n for n in ns if n > ndev]
        if skipped:
            print(f"# skipping N={skipped}: only {ndev} GPU(s) visible", file=sys.stderr)
        ns = [n for n in ns if n <= ndev]
    if not ns:
        print("no runnable GPU counts", file=sys.stderr)
        return 2
    bench_args = rest + (["--cpu"] if a.cpu else [])
    results = []
    for n in ns:
        d = run_point(n, bench_args, a.timeout)
        print(json.dumps(d), flush=True)
        results.append(d)
    c = curve(results)
    line = json.dumps(c)
    print(line, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0 if all(p["replica_ok"] is not False for p in c["points"]) else 3


if __name__ == "__main__":
    sys.exit(main())
