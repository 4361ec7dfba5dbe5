#!/usr/bin/env python3
"""Module cold start: process start -> first inference of ``python -m kvedge_amd.module``.

The one leg of boot-to-ready (helm install -> edgeAgent up, 156-216 s on the
reference) that a GPU box without a cluster can run.  The module is started as the guest
runs it (stdout transport instead of edgeHub), twice on the same fresh tuner cache file:

  cold: no tuner cache (first boot of a VM: every conv tile is timed)
  warm: the cache the first run wrote (every later boot: no tile sweep)

Each run writes the module's boot-timing stamps (the same file format as the guest's
/var/lib/kvedge/boot-timing) and the phase split is taken from them:

  import   process start (kernel start time) -> torch + op library + module imported
  model    imported -> ResNet-50 / YOLOv8n built (random init, BN folded, on the GPU)
  tune     -> conv tiles pinned (timed sweep, or read from the cache)
  warmup   -> warm-up steps
  capture  -> hipGraph captured
  graph_refine -> runner-up tiles A/B-timed in the captured step (engine.autotune.graph_refine;
           nothing to try when the tiles came from the cache)
  first    -> first inference finished

  python tools/module_cold_start.py --model resnet50 --batch 64 --out gpurun_out/cold.json
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEGS = [("import", "module_process_start", "module_imported"),
        ("model", "module_imported", "module_model_built"),
        ("tune", "module_model_built", "module_tuned"),
        ("warmup", "module_tuned", "module_warm"),
        ("capture", "module_warm", "module_graph_captured"),
        ("graph_refine", "module_graph_captured", "module_graph_refined"),
        ("first", "module_graph_refined", "module_first_inference")]


def one_run(model, batch, steps, work, cache, tag):
    stamps = os.path.join(work, f"stamps-{tag}")
    cmd = [sys.executable, "-m", "kvedge_amd.module", "--transport", "stdout",
           "--model", model, "--batch", str(batch), "--steps", str(steps),
           "--report-interval-s", "3600", "--state", os.path.join(work, f"state-{tag}.json"),
           "--stamps", stamps, "--tune-cache", cache]
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900)
    wall = time.time() - t0
    if r.returncode != 0:
        raise SystemExit(f"{tag}: module exited {r.returncode}\n{r.stderr[-3000:]}")
    st = {}
    for ln in open(stamps).read().splitlines():
        p = ln.split()
        if len(p) >= 2 and p[0] not in st:
            st[p[0]] = float(p[1])
    legs = {name: round(st[b] - st[a], 3) for name, a, b in LEGS if a in st and b in st}
    total = st["module_first_inference"] - st["module_process_start"]
    return {"run": tag, "start_to_first_inference_s": round(total, 3), "legs_s": legs,
            "spawn_to_exit_s": round(wall, 3),
            "tuner_cache": "hit" if tag == "warm" else "cold"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "yolov8n"])
    ap.add_argument("--batch", type=int, default=64, help="module twin batch (chart default 64)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as work:
        cache = os.path.join(work, "tune-cache.json")
        runs = [one_run(a.model, a.batch, a.steps, work, cache, "cold")]
        if not os.path.exists(cache):
            raise SystemExit("the cold run wrote no tuner cache")
        runs.append(one_run(a.model, a.batch, a.steps, work, cache, "warm"))
    res = {"what": "module process start -> first inference (python -m kvedge_amd.module, "
                   "stdout transport), one fresh MI355X box",
           "model": a.model, "batch": a.batch, "runs": runs}
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
