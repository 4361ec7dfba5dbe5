"""The kvedge IoT Edge module: twin-driven GPU inference with telemetry.

Plays the role SimulatedTemperatureSensor plays in the reference demo (cast :3524),
but the workload is ResNet-50 / YOLOv8n on the passed-through MI355X:

  start():   connect, read twin desired properties -> ModuleConfig, build the model +
             hipGraph engine, report effective config, resume counters from the state
             file on the persistent disk (checkpoint/resume).
  step():    one engine step (synthetic frames -> model) ; every report_interval_s a
             telemetry message on output "telemetry": images/sec, p50/p99 batch latency,
             cumulative images, top-1 histogram (ResNet) / detections (YOLO), heartbeat.
             With world_size > 1 the throughput counters are all-reduced over RCCL (C2)
             and rank 0 reports the job total.
  twin patch: validated; engine rebuilt only if a REBUILD key changed; reported props
             updated; invalid patches are rejected and reported, never crash the loop.
  direct methods: benchmark {steps, warmup}, getStatus, reconfigure {...}, ping.
  model "simulated-temperature": the reference demo's CPU-only plumbing workload
             (BASELINE config 1) -- machine/ambient temperature/pressure/humidity.
"""
from __future__ import annotations

import json
import math
import os
import random
import time
from typing import Any, Dict, Optional, Tuple

import torch

from .. import ops, parallel
from .config import ModuleConfig
from .transport import Transport, now_iso


class _SimTempModel:
    """SimulatedTemperatureSensor-compatible signal generator (CPU only)."""

    def __init__(self, seed: int):
        self.rng = random.Random(seed)
        self.t = 0

    def sample(self) -> Dict[str, Any]:
        self.t += 1
        machine_t = 21.0 + 0.2 * self.t + self.rng.uniform(-0.5, 0.5)
        return {"machine": {"temperature": round(machine_t, 3),
                            "pressure": round(1.0 + 0.1 * (machine_t - 21.0), 3)},
                "ambient": {"temperature": round(21.0 + self.rng.uniform(-0.5, 0.5), 3),
                            "humidity": round(24 + self.rng.uniform(0, 3), 1)},
                "timeCreated": now_iso()}


class _CameraSource:
    """Host frame producer for source="camera": cycles a few pre-rendered uint8 batches
    into a pinned FrameRing (drop-oldest when paced and the GPU falls behind), at ``fps``
    frames/s (0 = as fast as the ring drains).  Stands in for a camera / RTSP decoder
    thread; the hand-off path (pinned ring -> DMA in the native serve loop) is the
    production one."""

    def __init__(self, ring, batch: int, hw: int, fps: float, seed: int):
        import threading

        g = torch.Generator().manual_seed(seed)
        self.frames = [torch.randint(0, 256, (batch, hw, hw, 3), dtype=torch.uint8, generator=g)
                       for _ in range(3)]
        self.ring, self.batch, self.fps = ring, batch, fps
        self.seq = 0
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._run, name="kvedge-camera", daemon=True)
        self.thread.start()

    def _run(self):
        period = self.batch / self.fps if self.fps > 0 else 0.0
        nxt = time.perf_counter()
        while not self._stop.is_set():
            if not self.ring.put(self.frames[self.seq % len(self.frames)], self.seq,
                                 timeout_ms=100, drop_oldest=period > 0):
                continue
            self.seq += 1
            if period:
                nxt += period
                time.sleep(max(0.0, nxt - time.perf_counter()))

    def stop(self):
        self._stop.set()
        self.ring.close()
        self.thread.join(timeout=5)


class ModuleApp:
    def __init__(self, transport: Transport, config: Optional[ModuleConfig] = None,
                 device: Optional[str] = None, state_path: Optional[str] = None,
                 clock=time.perf_counter):
        self.tr = transport
        self.cfg = (config or ModuleConfig()).validate()
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.state_path = state_path
        self.clock = clock
        self.engine = None
        self.model = None
        self.ring = None
        self.camera: Optional[_CameraSource] = None
        self.sim: Optional[_SimTempModel] = None
        self.state = {"total_images": 0, "total_steps": 0, "restarts": 0, "rebuilds": 0,
                      "rejected_patches": 0, "messages": 0}
        self._win_imgs = 0
        self._win_t0 = 0.0
        self._lat_ms = []
        # native log-linear histogram (csrc/runtime): replicas merge it with one SUM
        # all-reduce, so the reported p99 is the fleet's true p99, not a max of p99s.
        # (device != cuda and no built library: plain list, CPU tests only)
        self._hist = None
        if self.device.type == "cuda" or ops.load():
            from ..runtime import LatencyHistogram

            self._hist = LatencyHistogram()
        self._last_report = 0.0
        self.last_telemetry: Optional[Dict[str, Any]] = None
        self.rank = parallel.info().rank
        self.world = parallel.info().world_size

    # ---------------------------------------------------------------- lifecycle
    def start(self):
        self.tr.set_twin_patch_handler(self.on_twin_patch)
        self.tr.set_method_handler(self.on_method)
        self.tr.connect()
        desired = self.tr.get_desired()
        try:
            self.cfg = self.cfg.apply_patch(desired)
        except (ValueError, TypeError) as e:
            self.state["rejected_patches"] += 1
            self.tr.patch_reported({"lastError": f"invalid desired properties: {e}"})
        self._load_state()
        self._build()
        self._report_config()
        self._win_t0 = self._last_report = self.clock()
        return self

    def stop(self):
        self._stop_camera()
        self._save_state()
        self.tr.disconnect()

    def _stop_camera(self):
        if self.camera is not None:
            self.camera.stop()
        self.camera = None
        self.ring = None

    def _load_state(self):
        if self.state_path and os.path.exists(self.state_path):
            try:
                with open(self.state_path) as f:
                    old = json.load(f)
                for k in ("total_images", "total_steps", "restarts", "rebuilds", "messages"):
                    self.state[k] = int(old.get(k, 0))
                self.state["restarts"] += 1
            except (OSError, ValueError):
                pass

    def _save_state(self):
        if not self.state_path:
            return
        os.makedirs(os.path.dirname(self.state_path) or ".", exist_ok=True)
        tmp = self.state_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(dict(self.state, config=self.cfg.to_dict(), ts=now_iso()), f)
        os.replace(tmp, self.state_path)  # atomic on the persistent disk

    def _build(self):
        cfg = self.cfg
        self._stop_camera()
        self.engine = None
        self.model = None
        self.sim = None
        if cfg.model == "simulated-temperature":
            self.sim = _SimTempModel(cfg.seed)
            return
        from ..engine import InferenceEngine

        dev = self.device
        if cfg.model == "resnet50":
            from ..models.resnet import KvResNet50

            self.model = KvResNet50.build(seed=cfg.seed, device=dev,
                                          calibrate=dev.type == "cuda")
        else:
            from ..models.yolov8 import KvYoloV8n, init_yolov8n

            self.model = KvYoloV8n(init_yolov8n(cfg.seed, calibrate=dev.type == "cuda"), dev,
                                   conf=cfg.conf, iou=cfg.iou, max_det=cfg.max_det)
        if self.world > 1:
            parallel.broadcast_tensors(parallel.model_tensors(self.model), src=0)
        camera = cfg.source == "camera"
        self.engine = InferenceEngine(self.model, cfg.batch, cfg.resolved_image_size(), device=dev,
                                      seed=cfg.seed + self.rank, use_graph=cfg.use_graph,
                                      synthetic=not camera)
        self.engine.prepare(warmup=1, autotune=dev.type == "cuda")
        if camera:
            from ..runtime import FrameRing

            self.ring = FrameRing(3, self.engine.frames.numel())
            self.camera = _CameraSource(self.ring, cfg.batch, cfg.resolved_image_size(), cfg.fps,
                                        cfg.seed + self.rank)

    def _report_config(self):
        self.tr.patch_reported({"config": self.cfg.to_dict(), "status": "running",
                                "device": str(self.device), "rank": self.rank,
                                "world_size": self.world, "restarts": self.state["restarts"]})

    # ---------------------------------------------------------------- main loop
    def step(self) -> None:
        self.tr.poll()
        if self.sim is not None:
            self._sim_step()
            return
        native = (self.cfg.native_loop and self.engine.graph is not None and
                  self._hist is not None)
        t0 = self.clock()
        if native:
            # C++ serve loop: per-step device time straight into the histogram; with a
            # camera source each replay first DMAs one pinned batch from the ring
            r = self.engine.serve_native(self.cfg.steps_per_poll, depth=2, hist=self._hist,
                                         ring=self.ring, ring_timeout_ms=1000)
            nsteps = r.steps
        else:
            if self.ring is not None:  # host path: take one ring batch, feed it, release
                slot, _ = self.ring.acquire_read(1000)
                if slot >= 0:
                    self.engine.frames.copy_(self.ring.slot(slot).view(self.engine.frames.shape))
                    self.ring.release(slot)
            self.engine.run()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            nsteps = 1
        dt = self.clock() - t0
        if not native:
            if self._hist is not None:
                self._hist.add_ms(dt * 1e3)
            else:
                self._lat_ms.append(dt * 1e3)
        self._win_imgs += self.cfg.batch * nsteps
        self.state["total_images"] += self.cfg.batch * nsteps
        self.state["total_steps"] += nsteps
        if self.cfg.fps > 0 and self.ring is None:
            budget = self.cfg.batch / self.cfg.fps
            if dt < budget:
                time.sleep(budget - dt)
        if self.clock() - self._last_report >= self.cfg.report_interval_s:
            self.report()

    def _sim_step(self):
        now = self.clock()
        if now - self._last_report >= self.cfg.send_interval_s or self.state["messages"] == 0:
            if self.state["messages"] < self.cfg.max_messages:
                self.tr.send_message("temperatureOutput", self.sim.sample())
                self.state["messages"] += 1
                self._last_report = now
                self._save_state()

    def run(self, max_steps: Optional[int] = None, duration_s: Optional[float] = None):
        t_end = None if duration_s is None else self.clock() + duration_s
        n = 0
        while (max_steps is None or n < max_steps) and (t_end is None or self.clock() < t_end):
            self.step()
            n += 1
        return n

    def _summary(self) -> Dict[str, Any]:
        now = self.clock()
        win = max(now - self._win_t0, 1e-9)
        ips = self._win_imgs / win
        if self._hist is not None:
            p50, p99 = self._hist.quantiles_us([0.5, 0.99])
            return {"images_per_s": ips, "p50_ms": p50 / 1e3, "p99_ms": p99 / 1e3,
                    "window_s": win, "steps": self._hist.count}
        lat = sorted(self._lat_ms)
        q = lambda p: lat[min(len(lat) - 1, int(round(p / 100 * (len(lat) - 1))))] if lat else 0.0  # noqa
        return {"images_per_s": ips, "p50_ms": q(50), "p99_ms": q(99), "window_s": win,
                "steps": len(lat)}

    def report(self) -> Dict[str, Any]:
        s = self._summary()
        ips_total, lat_max = s["images_per_s"], s["p99_ms"]
        if self.world > 1:  # C2 + C3 off the hot path, once per report interval
            ips_total = parallel.allreduce_scalars([s["images_per_s"]], op="sum")[0]
            if self._hist is not None:  # fleet p99 from the merged histogram
                self._hist.allreduce()
                lat_max = self._hist.quantiles_us([0.99])[0] / 1e3
            else:
                lat_max = parallel.allreduce_scalars([s["p99_ms"]], op="max")[0]
        msg = {"ts": now_iso(), "model": self.cfg.model, "batch": self.cfg.batch,
               "dtype": self.cfg.dtype, "images_per_s": round(ips_total, 2),
               "images_per_s_rank": round(s["images_per_s"], 2),
               "latency_ms": {"p50": round(s["p50_ms"], 3), "p99": round(lat_max, 3)},
               "total_images": self.state["total_images"], "rank": self.rank,
               "world_size": self.world, "heartbeat": self.state["total_steps"],
               "source": self.cfg.source}
        if self.ring is not None:
            msg["frames_dropped"] = self.ring.dropped
        msg.update(self._outputs_summary())
        if self.rank == 0:
            self.tr.send_message("telemetry", msg)
            self.state["messages"] += 1
        self.last_telemetry = msg
        self._win_imgs, self._lat_ms = 0, []
        if self._hist is not None:
            self._hist.reset()
        self._win_t0 = self._last_report = self.clock()
        self._save_state()
        return msg

    def _outputs_summary(self) -> Dict[str, Any]:
        out = self.engine.outputs if self.engine is not None else None
        if out is None:
            return {}
        if self.cfg.model == "resnet50":
            top1 = out[1].to("cpu")
            vals, counts = torch.unique(top1, return_counts=True)
            order = counts.argsort(descending=True)[:5]
            return {"top1": {str(int(vals[i])): int(counts[i]) for i in order}}
        dets, cnt = out
        cnt = cnt.to("cpu")
        return {"detections": {"total": int(cnt.sum()), "max_per_image": int(cnt.max())}}

    # ---------------------------------------------------------------- handlers
    def on_twin_patch(self, patch: Dict[str, Any]):
        try:
            new = self.cfg.apply_patch(patch)
        except (ValueError, TypeError) as e:
            self.state["rejected_patches"] += 1
            self.tr.patch_reported({"lastError": f"rejected patch: {e}"})
            return
        rebuild = new.needs_rebuild(self.cfg)
        self.cfg = new
        if rebuild:
            self.state["rebuilds"] += 1
            self._build()
        self._report_config()

    def on_method(self, name: str, payload: Dict[str, Any]) -> Tuple[int, Dict[str, Any]]:
        try:
            if name == "ping":
                return 200, {"pong": now_iso()}
            if name == "getStatus":
                return 200, {"config": self.cfg.to_dict(), "state": dict(self.state),
                             "last_telemetry": self.last_telemetry}
            if name == "reconfigure":
                self.on_twin_patch(payload)
                return 200, {"config": self.cfg.to_dict()}
            if name == "benchmark":
                if self.engine is None:
                    return 400, {"error": "no inference engine for model " + self.cfg.model}
                steps = int(payload.get("steps", 20))
                warm = int(payload.get("warmup", 3))
                for _ in range(warm):
                    self.engine.run()
                dt = self.engine.run_timed(steps)
                lat = self.engine.measure_latency(min(steps, 20))
                ips = steps * self.cfg.batch / dt
                if self.world > 1:
                    ips = parallel.allreduce_scalars([ips], op="sum")[0]
                return 200, {"images_per_s": round(ips, 2), "steps": steps,
                             "batch": self.cfg.batch, "p50_ms": round(lat.percentile(50), 3),
                             "p99_ms": round(lat.percentile(99), 3)}
            return 404, {"error": f"unknown method {name}"}
        except Exception as e:  # a bad method call must not kill the module
            return 500, {"error": repr(e)}
