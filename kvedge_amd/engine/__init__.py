"""N16 inference engine: static shapes, on-device synthetic frames, one hipGraph per forward.

The whole edge-module step (K11 frame synthesis -> preprocess -> model -> softmax/
top-1, or -> YOLO decode -> NMS) is captured once with ``torch.cuda.CUDAGraph``
(which IS hipGraph on ROCm) and replayed per batch: launch overhead of ~60
kernels collapses to one graph launch (MI355X_MICROARCH.md price row
"graph-replay-floor").  The frame counter lives in device memory and is bumped
inside the graph, so every replay sees fresh frames.

On CPU the same engine runs the reference path eagerly (tests, no GPU).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

from .. import ops

# Per-GPU batch bench.py times by default (and tests/test_bench_config_gpu.py checks).
# ResNet-50: 1280, from the same-box batch sweeps (profiles/r2_v8_batch_sweep.jsonl):
# 79.6-80.3k img/s at 1280 against 78.1-78.2k at 640, the largest batch whose activations
# still fit one launch per conv (2 GiB per operand; ~1330 images); re-checked on the round-4
# tree (profiles/r4_v7_resnet50_batch_recheck.md).  YOLOv8n: 512, from the round-4 same-box
# re-check (profiles/r4_v7_yolov8n_batch_recheck.md: 46.5-46.8k against 45.9-46.0k at 384;
# 384 was round 1's sweep knee).  Edge-module serving uses its own, latency-bound batch
# (module twin `batch`, default 64).
BENCH_BATCH = {"resnet50": 1280, "yolov8n": 512}
# Batch slices per step, each on its own HIP stream (parallel branches of one hipGraph).
# Two slices run concurrently fill each other's kernel drain/fill bubbles (same-box A/B,
# profiles/r2_v17_streams_ab.jsonl): ResNet-50 b1280 75.4k -> 79.9k img/s, YOLOv8n b384
# 38.4k -> 39.8k.  3-4 slices, or slices phase-shifted by event dependencies, lose
# (profiles/r2_v17_stream_probe.jsonl).
BENCH_STREAMS = {"resnet50": 2, "yolov8n": 2}


@dataclass
class StepTimes:
    count: int = 0
    total_s: float = 0.0
    samples_ms: List[float] = field(default_factory=list)

    def add(self, dt_s: float, keep: int = 4096):
        self.count += 1
        self.total_s += dt_s
        if len(self.samples_ms) < keep:
            self.samples_ms.append(dt_s * 1e3)

    def percentile(self, q: float) -> float:
        if not self.samples_ms:
            return 0.0
        s = sorted(self.samples_ms)
        i = min(len(s) - 1, max(0, int(round(q / 100.0 * (len(s) - 1)))))
        return s[i]


def _cat_outputs(parts):
    """Per-slice model outputs (a tensor or a tuple of tensors) -> full-batch outputs."""
    if isinstance(parts[0], torch.Tensor):
        return torch.cat(parts, 0)
    return tuple(torch.cat(xs, 0) for xs in zip(*parts))


class InferenceEngine:
    """Runs ``model(frames_u8) -> outputs`` on static-shape batches.

    model: any callable taking a uint8 NHWC3 frame batch (KvResNet50, KvYoloV8n).
    streams: split each step's batch into this many equal slices, each run by the model on
    its own HIP stream (forked from and joined back into the step's stream, so one hipGraph
    holds them as parallel branches); per-slice outputs are concatenated along the batch.
    """

    def __init__(self, model: Callable, batch: int, image_size: int, device="cuda",
                 seed: int = 0, use_graph: bool = True, synthetic: bool = True,
                 streams: int = 1):
        self.model = model
        self.batch = batch
        self.hw = image_size
        self.device = torch.device(device)
        self.seed = seed
        self.use_graph = use_graph and self.device.type == "cuda"
        # synthetic=False: the graph reads self.frames as-is (fed by set_frames, or by
        # the native serve loop from a pinned FrameRing -- kvedge_amd.runtime)
        self.synthetic = synthetic
        self.frames = torch.empty(batch, image_size, image_size, 3, dtype=torch.uint8,
                                  device=self.device)
        # [step counter, finished-block count]: synth_frames bumps it in-kernel (one launch)
        self.step_ctr = torch.zeros(2, dtype=torch.int64, device=self.device)
        self.outputs = None
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.times = StepTimes()
        if streams < 1 or batch % streams:
            raise ValueError(f"batch {batch} does not split into {streams} equal slices")
        self.n_streams = streams if self.device.type == "cuda" else 1
        # KVEDGE_STREAM_PRIO=1: the first slice's stream at high priority, the others normal
        # (the dispatcher then feeds slice 0's workgroups first and the others fill the CUs
        # its kernels leave idle) -- an A/B knob, off by default
        prio = os.environ.get("KVEDGE_STREAM_PRIO", "0") == "1"
        self._side = [torch.cuda.Stream(device=self.device, priority=-1 if (prio and i == 0) else 0)
                      for i in range(self.n_streams)] if self.n_streams > 1 else []

    # one full edge-module step: synthesize frames, run the model
    def _step(self):
        if self.synthetic:
            ops.synth_frames(self.frames, self.seed, self.step_ctr)
        return self._forward()

    def _forward(self):
        if not self._side:
            self.outputs = self.model(self.frames)
            return self.outputs
        cur = torch.cuda.current_stream(self.device)
        per = self.batch // self.n_streams
        parts = []
        for i, s in enumerate(self._side):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                parts.append(self.model(self.frames[i * per:(i + 1) * per]))
        for s in self._side:
            cur.wait_stream(s)
        self.outputs = _cat_outputs(parts)
        return self.outputs

    def prepare(self, warmup: int = 2, autotune: bool = True, verbose: bool = False,
                tune_cache: Optional[str] = None, refine_s: Optional[float] = None):
        """Autotune conv tiles for this batch, warm up (code objects load, allocator
        pools fill), then capture the step into a hipGraph.  ``tune_cache``: JSON file of
        earlier picks (autotune.autotune), so a restarted module skips the timing sweep.
        ``self.prep_s`` keeps the phase times (tune / warmup / capture).  ``refine_s``: budget
        of the in-graph tile refinement (None = KVEDGE_GRAPH_REFINE_S, default 0 = off: on
        four fresh boxes it kept at most one swap for a net -0.5 .. +0.1 %, VERDICT r5
        weak #4, so it is opt-in; when on it verifies its result against the original
        capture before committing)."""
        self.tuning = {}
        self.prep_s = {}
        t0 = time.perf_counter()
        if autotune and self.device.type == "cuda":
            from .autotune import autotune as _tune

            ops.synth_frames(self.frames, self.seed, 0)
            # tiles are pinned per layer for the shape the model actually runs: one slice
            conc = self.n_streams if os.environ.get("KVEDGE_TUNE_CONCURRENT", "1") != "0" else 1
            self.tuning = _tune(self.model, self.frames[:self.batch // self.n_streams],
                                verbose=verbose, concurrency=conc, cache_path=tune_cache)
            if tune_cache:
                # an earlier engine of this batch x streams refined tiles in its graph
                from .autotune import apply_refined

                self.refined_from_cache = apply_refined(self, tune_cache)
            torch.cuda.synchronize(self.device)
        t1 = time.perf_counter()
        self.prep_s["tune"] = t1 - t0
        if not self.use_graph:
            for _ in range(warmup):
                self._step()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.prep_s["warmup"] = time.perf_counter() - t1
            return self
        self._cap_stream = s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(max(1, warmup)):
                self._step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        t2 = time.perf_counter()
        self.prep_s["warmup"] = t2 - t1
        self.graph, self.outputs = self.capture(warm=False)
        self.prep_s["capture"] = time.perf_counter() - t2
        self.refine = None
        if refine_s is None:
            refine_s = float(os.environ.get("KVEDGE_GRAPH_REFINE_S", "0"))
        if (autotune and self.tuning and refine_s > 0 and
                os.environ.get("KVEDGE_GRAPH_REFINE", "1") != "0"):
            # in-graph pick of the tiles (autotune.graph_refine): per-layer timing alone
            # does not see the neighbouring layers and the other slice's kernels
            from .autotune import graph_refine

            t3 = time.perf_counter()
            self.refine = graph_refine(self, budget_s=refine_s, verbose=verbose,
                                       cache_path=tune_cache)
            self.prep_s["graph_refine"] = time.perf_counter() - t3
        return self

    def capture(self, warm: bool = True):
        """Capture one step (with the layers' current tiles) into a new hipGraph; returns
        (graph, its output tensors).  ``self.graph`` is not touched.  ``warm``: one eager step first on the capture
        stream (validates the tiles, creates per-stream state such as the split-K
        workspace outside the capture)."""
        s = self._cap_stream
        if warm:
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._step()
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        # capture on the warm-up stream: per-stream state made during warm-up (the split-K
        # workspace, ops.splitk_workspace) is then reused, not re-allocated -- and zero-filled
        # by a kernel recorded into the graph, i.e. on every replay -- for a new stream
        with torch.cuda.graph(g, stream=s):
            self._step()
        torch.cuda.synchronize(self.device)
        return g, self.outputs  # the outputs live in this graph's private pool

    def run(self):
        """Launch one step (async on GPU)."""
        if self.graph is not None:
            self.graph.replay()
        else:
            self._step()
        return self.outputs

    def run_timed(self, n: int) -> float:
        """Run n steps, return elapsed seconds (device-synchronised)."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        for _ in range(n):
            self.run()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - t0
        return dt

    def measure_latency(self, n: int) -> StepTimes:
        """Per-step latency with a sync after every step (p50/p99 telemetry)."""
        st = StepTimes()
        for _ in range(n):
            dt = self.run_timed(1)
            st.add(dt)
        return st

    def serve_native(self, n_steps: int, depth: int = 2, hist=None, ring=None,
                     ring_timeout_ms: int = 1000):
        """Replay the captured step ``n_steps`` times from the native C++ loop
        (csrc/runtime: no Python per step, per-step device time into ``hist``).  With a
        FrameRing, each step first DMAs one pinned frame batch into ``self.frames``
        (build the engine with synthetic=False so the graph does not overwrite them)."""
        from .. import runtime

        if self.graph is None:
            raise RuntimeError("serve_native needs a captured graph (prepare() on a GPU)")
        if ring is not None and self.synthetic:
            raise ValueError("ring-fed serving needs InferenceEngine(synthetic=False)")
        with torch.cuda.device(self.device):
            return runtime.serve(self.graph, n_steps, depth=depth, hist=hist, ring=ring,
                                 dev_input=self.frames if ring is not None else None,
                                 ring_timeout_ms=ring_timeout_ms)

    def memory_plan(self, align: int = 256):
        """Native arena plan of one step's activations (kvedge_amd.runtime.plan_memory)."""
        from .. import runtime

        return runtime.plan_memory(lambda: self.model(self.frames), self.batch, align)

    def set_frames(self, frames_u8: torch.Tensor):
        """Feed real frames instead of synthetic (disables the synthetic step)."""
        self.frames.copy_(frames_u8)
        return self._forward()


def edge_streams(batch: int) -> int:
    """Batch slices (HIP streams) for a serving batch: one.  Two half-batch slices on two
    streams were measured SLOWER at the serving sizes on the same box (b32 0.95 vs 0.87 ms,
    b64 1.41 vs 1.30 ms p50, profiles/r3_v11_edge_streams_ab.txt): at these sizes the
    half-batch kernels lose more to their own launch floors than the overlap recovers.
    KVEDGE_EDGE_STREAMS=n overrides (n must divide the batch)."""
    env = os.environ.get("KVEDGE_EDGE_STREAMS", "")
    if env:
        n = int(env)
        return n if n >= 1 and batch % n == 0 else 1
    return 1


def edge_latency(model: Callable, image_size: int, batches, device="cuda", seed: int = 0,
                 steps: int = 200, warmup: int = 20) -> List[Dict[str, float]]:
    """Edge-serving operating points (module twin ``batch``, default 64): per batch size a
    fresh single-stream engine (tiles autotuned for THAT batch, one hipGraph), then
    ``steps`` replays each followed by a device sync -- the latency a module step sees.
    Run it after any headline timing: it re-pins the model's conv tiles."""
    out = []
    for b in batches:
        eng = InferenceEngine(model, b, image_size, device=device, seed=seed, use_graph=True,
                              streams=edge_streams(b))
        eng.prepare(warmup=2, autotune=True)
        for _ in range(warmup):
            eng.run()
        st = eng.measure_latency(steps)
        p50, p99 = st.percentile(50), st.percentile(99)  # ms
        out.append({"batch": b, "streams": eng.n_streams, "p50_ms": round(p50, 4),
                    "p99_ms": round(p99, 4),
                    "images_per_s": round(b / (p50 / 1e3), 1), "steps": steps})
        del eng
    return out
