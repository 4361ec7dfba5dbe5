#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 bf16 edge-module inference images/sec on 1..8 MI355X.

Metric/config are the ones BASELINE.json names ("images/sec ResNet-50 edge module at
1/2/4/8 MI355X").  One step = one full edge-module step on every GPU:
on-device synthetic uint8 frames (K11) -> preprocess (K12) -> ResNet-50 forward
(hand-written gfx950 HIP kernels) -> softmax + top-1, captured in one hipGraph.
Weights are random-init (seeded) ResNet-50 v1.5 of the full architecture.

Data parallel, weak scaling: each rank runs its own per-GPU batch; the value is the
WHOLE-JOB images/sec = world * batch * steps / max_rank_elapsed.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
  torchrun --nproc-per-node N bench.py --gpus N ...

Without a launcher (no WORLD_SIZE in the env) ``--gpus N>1`` makes this process a
launcher: it counts devices (no HIP initialisation), spawns N fresh ranks of itself
with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, and exits with the first failing rank's
code.  After the timed loop every rank replays one batch of frames from a SHARED seed
and the ranks compare digests of the pre-softmax logits (C4): a replica whose
weights or kernels drifted fails the run instead of silently skewing it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec ResNet-50 edge module at 1/2/4/8 MI355X; VM boot-to-ready sec"
# per-model metric strings: only the ResNet-50 run is BASELINE.json's headline
METRICS = {"resnet50": METRIC,
           "yolov8n": "images/sec YOLOv8n detection edge module (incl. decode + NMS) on MI355X"}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("KVEDGE_BENCH_BATCH", 0)),
                    help="per-GPU batch (0 = kvedge_amd.engine.BENCH_BATCH: ResNet-50 1280, "
                         "YOLOv8n 512, from the batch sweeps in profiles/)")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "yolov8n"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--streams", type=int, default=int(os.environ.get("KVEDGE_STREAMS", 0)),
                    help="batch slices per step, one HIP stream each (0 = per-model default, "
                         "engine.BENCH_STREAMS)")
    ap.add_argument("--no-autotune", action="store_true")
    ap.add_argument("--microbatch", type=int, default=int(os.environ.get("KVEDGE_MICROBATCH", 0)),
                    help="ResNet-50: run the first --mb-blocks bottlenecks in micro-batches "
                         "(Infinity-Cache residency); 0 = off")
    ap.add_argument("--mb-blocks", type=int, default=int(os.environ.get("KVEDGE_MB_BLOCKS", 3)))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--profile", default=None, metavar="PATH",
                    help="after the timed run, profile one eager step per op (HIP events) "
                         "and write the per-call table as JSON to PATH (rank 0)")
    ap.add_argument("--cpu", action="store_true",
                    help="plumbing check only: run the same DP bench path on the CPU "
                         "reference ops over gloo (tests/test_bench_cpu.py); not a measurement")
    ap.add_argument("--native-loop", action="store_true",
                    help="time the K steps with the native C++ serve loop (csrc/runtime) "
                         "instead of Python graph.replay() calls")
    ap.add_argument("--launch-timeout", type=float,
                    default=float(os.environ.get("KVEDGE_LAUNCH_TIMEOUT", 1500)),
                    help="self-launch (--gpus N > 1 without torchrun): kill every rank after "
                         "this many seconds (a hung RCCL init must not hang the job)")
    ap.add_argument("--edge", default=os.environ.get("KVEDGE_EDGE", "1,8,64"),
                    help="ResNet-50: after the headline (untimed for it), p50/p99 latency at "
                         "these edge batch sizes -> extra.edge ('' = skip)")
    ap.add_argument("--yolo", type=int, default=int(os.environ.get("KVEDGE_BENCH_YOLO", 1)),
                    help="ResNet-50 run: after the headline and the edge block (untimed for "
                         "them), also time YOLOv8n + decode + NMS at its bench config "
                         "(engine.BENCH_BATCH / BENCH_STREAMS) -> extra.yolov8n (0 = skip)")
    ap.add_argument("--perturb-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--hang-rank", type=int, default=-1, help=argparse.SUPPRESS)
    raw = list(sys.argv[1:] if argv is None else argv)
    a = ap.parse_args(raw)

    from kvedge_amd import parallel

    if a.gpus < 1:
        print("--gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # launcher path: no torch.cuda.* call may run here (HIP would initialise in the
        # parent of the GPU ranks); devices are counted from the KFD topology in sysfs
        if not a.cpu:
            ndev = parallel.visible_gpu_count()
            if a.gpus > ndev:
                print(f"--gpus {a.gpus} but only {ndev} GPU(s) visible", file=sys.stderr)
                return 2
        return parallel.launch_local(a.gpus, [os.path.abspath(__file__)] + raw,
                                     timeout_s=a.launch_timeout if a.launch_timeout > 0 else None)
    if int(os.environ.get("WORLD_SIZE", "1")) != a.gpus:
        print(f"# note: --gpus {a.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')}; "
              "reporting the launched world size", file=sys.stderr)

    import torch
    from kvedge_amd import ops
    from kvedge_amd.engine import BENCH_BATCH, BENCH_STREAMS, InferenceEngine

    if a.hang_rank >= 0 and a.hang_rank == int(os.environ.get("RANK", "0")):
        while True:  # test hook (tests/test_bench_cpu.py): a rank that never arrives
            time.sleep(3600)
    di = parallel.init_from_env(prefer_gpu=not a.cpu)
    on_gpu = di.device.type == "cuda"
    if not on_gpu and not a.cpu:
        print("bench.py needs a GPU (MI355X); none visible", file=sys.stderr)
        return 2
    if on_gpu and not ops.load():
        raise RuntimeError("kvedge native kernels not built: run python -m kvedge_amd._build")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    if a.batch <= 0:
        a.batch = BENCH_BATCH[a.model] if on_gpu else 1
    if a.streams <= 0:
        a.streams = BENCH_STREAMS[a.model] if on_gpu else 1
    if a.batch % a.streams:
        a.streams = 1
    t_build = time.perf_counter()
    if a.model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50

        model = KvResNet50.build(seed=a.seed, device=di.device, calibrate=on_gpu)
        model.microbatch, model.microbatch_blocks = a.microbatch, a.mb_blocks
        hw = KvResNet50.image_size
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n

        model = KvYoloV8n.build(seed=a.seed, device=di.device, calibrate=on_gpu)
        hw = KvYoloV8n.image_size
    # C1: every replica serves rank 0's weights
    parallel.broadcast_tensors(parallel.model_tensors(model), src=0)
    if a.perturb_rank == di.rank:  # test hook: a drifted replica must fail C4
        with torch.no_grad():
            parallel.model_tensors(model)[-1].add_(0.05)
    eng = InferenceEngine(model, a.batch, hw, device=di.device, seed=a.seed + di.rank,
                          use_graph=not a.no_graph, streams=a.streams)
    eng.prepare(warmup=2, autotune=not a.no_autotune)
    build_s = time.perf_counter() - t_build
    from kvedge_amd.utils.logging import get_logger, log_event

    log = get_logger("kvedge.bench")
    if di.is_main:
        log_event(log, "built", model=a.model, batch=a.batch, world=di.world_size,
                  build_s=round(build_s, 2), tuned_layers=len(getattr(eng, "tuning", {}) or {}))

    for _ in range(a.warmup):
        eng.run()
    sync()
    parallel.barrier()
    sync()
    lat_hist = None
    t0 = time.perf_counter()
    if a.native_loop and eng.graph is not None:
        from kvedge_amd.runtime import LatencyHistogram

        lat_hist = LatencyHistogram()
        eng.serve_native(a.steps, depth=2, hist=lat_hist)
    else:
        for _ in range(a.steps):
            eng.run()
    sync()
    elapsed = time.perf_counter() - t0
    parallel.barrier()
    sync()

    hip_graph, n_streams = eng.graph is not None, eng.n_streams
    # C3: job time = slowest rank
    (max_elapsed,) = parallel.allreduce_scalars([elapsed], op="max")
    # C4 (untimed): every rank runs the same frames (shared seed, not seed+rank) through
    # its own weights/kernels; digests of the pre-softmax outputs must agree
    with torch.no_grad():
        ops.synth_frames(eng.frames, a.seed, 0)
        raw_out = model.raw_outputs(eng.frames)
        local = parallel.digest(raw_out)
    sync()
    rc = parallel.check_replicas(local)
    del raw_out
    edge = None
    if on_gpu and a.model == "resnet50" and a.edge.strip():
        # the module's real operating points (twin batch, default 64), after the headline
        # timing and the C4 check so neither can be distorted by it
        from kvedge_amd.engine import edge_latency

        edge = edge_latency(model, hw, [int(b) for b in a.edge.split(",") if b.strip()],
                            device=di.device, seed=a.seed + di.rank)

    yolo = None
    if on_gpu and a.model == "resnet50" and a.yolo:
        # BASELINE.json config 4 under the same clock discipline as the headline: fresh
        # engine at its own bench config, W untimed warmup steps, K timed steps bracketed
        # by barrier + synchronize, slowest rank's time (the ResNet-50 engine stays
        # allocated: a few GB of 288)
        yolo = _time_yolo(a, di, sync)

    world = parallel.info().world_size
    imgs = world * a.batch * a.steps
    value = imgs / max_elapsed
    ms_per_step = max_elapsed / a.steps * 1e3
    flops = model.flops_per_image(hw) if hasattr(model, "flops_per_image") else None
    res = {
        "metric": METRICS[a.model],
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": ("synthetic (on-device uint8 frames), random-init seeded weights" if on_gpu
                 else "CPU plumbing check (reference ops) -- NOT a measurement"),
        "config": {
            "model": a.model,
            "global_batch": world * a.batch,
            "per_gpu_batch": a.batch,
            "seq_len": None,
            "image_size": hw,
            "parallelism": f"dp{world}",
            "backend": di.backend,
            "hip_graph": hip_graph,
            "streams": n_streams,
            "microbatch": getattr(model, "microbatch", 0),
            "mb_blocks": getattr(model, "microbatch_blocks", 0),
        },
        "extra": {
            "tflops_per_gpu": round(value / world * flops / 1e12, 2) if flops else None,
            "build_s": round(build_s, 2),
            "prepare_s": {k: round(v, 2) for k, v in (getattr(eng, "prep_s", None) or {}).items()},
            "graph_refine": getattr(eng, "refine", None),
            "replica_check": {"ok": rc.ok, "max_rel_dev": rc.max_rel_dev,
                              "digests": rc.digests},
            "backend": di.backend,
            "timed_loop": "native" if lat_hist is not None else "python",
        },
    }
    if edge is not None:
        res["extra"]["edge"] = edge
    if yolo is not None:
        res["extra"]["yolov8n"] = yolo
    if lat_hist is not None:
        lat_hist.allreduce()  # fleet-wide step-latency distribution (one SUM all-reduce)
        res["extra"]["step_latency_ms"] = {k: round(v, 4) for k, v in lat_hist.summary().items()}
    if di.is_main:
        log_event(log, "timed", steps=a.steps, ms_per_step=res["ms_per_step"],
                  value=res["value"], replica_ok=rc.ok)
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if a.profile and di.is_main:
        from kvedge_amd.engine.profile import write_profile

        prof = write_profile(eng, a.profile)
        top = list(prof["by_op_ms"].items())[:6]
        print(f"# eager-step profile -> {a.profile}: total {prof['total_ms']:.2f} ms; "
              + ", ".join(f"{k} {v:.2f}" for k, v in top), file=sys.stderr)
    parallel.shutdown()
    if not rc.ok:
        print(f"replica check FAILED: max relative deviation {rc.max_rel_dev:.3e} "
              f"(digests {rc.digests})", file=sys.stderr)
        return 3
    return 0


def _time_yolo(a, di, sync):
    """YOLOv8n (incl. decode + NMS) images/sec at engine.BENCH_BATCH["yolov8n"] per GPU with
    engine.BENCH_STREAMS["yolov8n"] slices: same W/K and timing rules as the headline."""
    import torch
    from kvedge_amd import parallel
    from kvedge_amd.engine import BENCH_BATCH, BENCH_STREAMS, InferenceEngine
    from kvedge_amd.models.yolov8 import KvYoloV8n

    torch.cuda.empty_cache()
    batch, streams = BENCH_BATCH["yolov8n"], BENCH_STREAMS["yolov8n"]
    t_build = time.perf_counter()
    model = KvYoloV8n.build(seed=a.seed, device=di.device, calibrate=True)
    parallel.broadcast_tensors(parallel.model_tensors(model), src=0)
    eng = InferenceEngine(model, batch, KvYoloV8n.image_size, device=di.device,
                          seed=a.seed + di.rank, use_graph=True, streams=streams)
    eng.prepare(warmup=2, autotune=True)
    build_s = time.perf_counter() - t_build
    for _ in range(a.warmup):
        eng.run()
    sync()
    parallel.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.run()
    sync()
    elapsed = time.perf_counter() - t0
    parallel.barrier()
    sync()
    (mx,) = parallel.allreduce_scalars([elapsed], op="max")
    world = parallel.info().world_size
    out = {"metric": METRICS["yolov8n"], "value": round(world * batch * a.steps / mx, 2),
           "ms_per_step": round(mx / a.steps * 1e3, 4), "per_gpu_batch": batch,
           "streams": eng.n_streams, "steps": a.steps, "warmup": a.warmup,
           "image_size": KvYoloV8n.image_size, "build_s": round(build_s, 2),
           "graph_refine": eng.refine}
    del eng, model
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    sys.exit(main())
