"""Edge-module configuration = IoT Edge module twin desired properties (SURVEY.md §5.6 layer 4).

The reference's config layers are Helm values -> cloud-init -> config.toml; the module
layer (IoT Hub deployment manifest + twin) is where the reference's demo module
(SimulatedTemperatureSensor) takes its settings.  kvedge keeps that shape: the twin's
desired properties below drive the GPU inference module, and the same keys exist as
CLI flags for bare-metal runs (kvedge_amd.module.__main__).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, fields, replace
from typing import Any, Dict

MODELS = ("resnet50", "yolov8n", "simulated-temperature")
SOURCES = ("synthetic", "camera")
DTYPES = ("bf16",)


@dataclass(frozen=True)
class ModuleConfig:
    model: str = "resnet50"
    batch: int = 64
    dtype: str = "bf16"
    seed: int = 0
    report_interval_s: float = 10.0
    world_size: int = 1
    image_size: int = 0          # 0 = model default (224 / 640)
    conf: float = 0.25           # YOLO score threshold
    iou: float = 0.7             # YOLO NMS IoU threshold
    max_det: int = 300
    fps: float = 0.0             # 0 = run flat out; > 0 throttles batches/s*batch
    use_graph: bool = True
    # frame source: "synthetic" = on-device generator inside the graph; "camera" = a host
    # producer thread feeding a pinned FrameRing that the native serve loop DMAs from
    source: str = "synthetic"
    native_loop: bool = True     # GPU: replay the graph from the C++ serve loop
    steps_per_poll: int = 1      # graph replays per module step (native loop)
    # seconds of in-graph tile refinement when the engine is built (engine.prepare refine_s;
    # 0 = off, the default).  It times runner-up tiles inside the captured step; on the
    # driver's fresh boxes it returned -0.5 .. +0.1 % (BENCH_r05 / r6 builder boxes) for
    # 3.1 s of a 6.6 s cold start, so it is opt-in
    refine_s: float = 0.0
    # multi-replica lockstep: module steps between control boundaries (0 = auto: every
    # step at world 1, 16 otherwise).  Twin patches, collective direct methods, report
    # decisions and stop requests are exchanged ONLY at these boundaries, so every rank
    # issues the same collectives in the same order.  Rank 0's value wins fleet-wide.
    sync_every: int = 0
    # SimulatedTemperatureSensor compatibility (BASELINE config 1, CPU-only plumbing)
    send_interval_s: float = 5.0
    max_messages: int = 500

    # keys that force an engine rebuild when they change
    REBUILD = ("model", "batch", "dtype", "seed", "image_size", "conf", "iou", "max_det",
               "use_graph", "source")

    def validate(self) -> "ModuleConfig":
        if self.model not in MODELS:
            raise ValueError(f"model must be one of {MODELS}, got {self.model!r}")
        if self.dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {DTYPES} (bf16 compute), got {self.dtype!r}")
        if not 1 <= self.batch <= 4096:
            raise ValueError(f"batch out of range: {self.batch}")
        if self.report_interval_s <= 0:
            raise ValueError("report_interval_s must be > 0")
        if not 1 <= self.world_size <= 64:
            raise ValueError("world_size must be 1..64")
        if self.image_size and self.image_size % 32:
            raise ValueError("image_size must be a multiple of 32")
        if not 0.0 <= self.conf <= 1.0 or not 0.0 <= self.iou <= 1.0:
            raise ValueError("conf/iou must be in [0, 1]")
        if not 1 <= self.max_det <= 300:
            raise ValueError("max_det must be 1..300")
        if self.source not in SOURCES:
            raise ValueError(f"source must be one of {SOURCES}, got {self.source!r}")
        if not 1 <= self.steps_per_poll <= 1000:
            raise ValueError("steps_per_poll must be 1..1000")
        if not 0.0 <= self.refine_s <= 600.0:
            raise ValueError("refine_s must be 0..600")
        if not 0 <= self.sync_every <= 10000:
            raise ValueError("sync_every must be 0..10000")
        return self

    def apply_patch(self, patch: Dict[str, Any]) -> "ModuleConfig":
        """Apply a (partial) twin desired-properties patch; unknown keys and the
        IoT Hub '$version' bookkeeping are ignored; types are coerced."""
        kw = {}
        by_name = {f.name: f for f in fields(self)}
        for k, v in (patch or {}).items():
            if k.startswith("$") or k not in by_name:
                continue
            cur = getattr(self, k)
            if isinstance(cur, bool):
                v = v if isinstance(v, bool) else str(v).lower() in ("1", "true", "yes")
            elif isinstance(cur, int):
                v = int(v)
            elif isinstance(cur, float):
                v = float(v)
            else:
                v = str(v)
            kw[k] = v
        return replace(self, **kw).validate()

    def needs_rebuild(self, other: "ModuleConfig") -> bool:
        return any(getattr(self, k) != getattr(other, k) for k in self.REBUILD)

    def resolved_image_size(self) -> int:
        if self.image_size:
            return self.image_size
        return 640 if self.model == "yolov8n" else 224

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)
