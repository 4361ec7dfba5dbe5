"""Python face of the native serving runtime (csrc/runtime/kv_runtime.{h,cpp}).

The reference (levi106/kvedge) has no serving runtime: the workload is whatever IoT Edge
module edgeAgent starts (cast :2890, :3524).  Here the in-guest module
(kvedge_amd/module) sits on a native C++ runtime:

* :class:`LatencyHistogram` -- log-linear latency histogram (3 % buckets) whose storage is
  a flat int64 tensor, so replicas merge with one all_reduce(SUM) and report fleet-wide
  p50/p99.
* :func:`plan_memory` -- records every activation allocation of one forward (lifetimes
  in op order), hands them to the native greedy-by-size arena planner and returns the
  per-image activation footprint; :func:`max_batch` sizes the per-GPU batch against
  288 GB of HBM3E.
* :class:`FrameRing` + :func:`serve` -- pinned host frame ring and the native hipGraph
  replay loop (no Python / GIL per step; steps in flight bounded by ``depth``).

Every entry point fails loudly when the native library is missing.
"""
from __future__ import annotations

import threading
import weakref
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import torch

from .. import ops

HBM_BYTES_MI355X = 288 * 10**9


def _k():
    if not ops.load():
        raise RuntimeError("kvedge_amd native runtime unavailable: build with "
                           "`python -m kvedge_amd._build`")
    return torch.ops.kvedge


# ---------------------------------------------------------------------------
# latency histogram
# ---------------------------------------------------------------------------
class LatencyHistogram:
    """Step-latency histogram (microseconds) backed by a CPU int64 tensor."""

    def __init__(self, data: Optional[torch.Tensor] = None):
        n = _k().hist_len()
        self.data = torch.zeros(n, dtype=torch.int64) if data is None else data
        if self.data.numel() != n:
            raise ValueError(f"histogram tensor must have {n} entries")

    def add(self, us: float) -> None:
        _k().hist_add(self.data, float(us))

    def add_many(self, us: Sequence[float]) -> None:
        _k().hist_add_many(self.data, torch.as_tensor(list(us), dtype=torch.float64))

    def add_ms(self, ms: float) -> None:
        self.add(ms * 1e3)

    @property
    def count(self) -> int:
        return int(self.data[-2])

    def mean_us(self) -> float:
        return float(_k().hist_mean(self.data))

    def quantiles_us(self, qs: Sequence[float]) -> List[float]:
        return list(_k().hist_quantiles(self.data, [float(q) for q in qs]))

    def percentile_ms(self, p: float) -> float:
        return self.quantiles_us([p / 100.0])[0] / 1e3

    def merge(self, other: "LatencyHistogram") -> "LatencyHistogram":
        self.data += other.data
        return self

    def reset(self) -> None:
        self.data.zero_()

    def allreduce(self) -> "LatencyHistogram":
        """Merge every replica's histogram in place (one SUM all-reduce)."""
        from .. import parallel

        if parallel.is_dist():
            import torch.distributed as dist

            dev = parallel.info().device
            t = self.data.to(dev)
            dist.all_reduce(t, dist.ReduceOp.SUM)
            self.data.copy_(t.cpu())
        return self

    def summary(self) -> dict:
        p50, p90, p99 = self.quantiles_us([0.5, 0.9, 0.99])
        return {"count": self.count, "mean_ms": self.mean_us() / 1e3, "p50_ms": p50 / 1e3,
                "p90_ms": p90 / 1e3, "p99_ms": p99 / 1e3}


# ---------------------------------------------------------------------------
# activation memory planning
# ---------------------------------------------------------------------------
@dataclass
class MemoryPlan:
    batch: int
    slab_bytes: int                 # arena size from the native planner
    live_peak_bytes: int            # max simultaneously-live bytes (lower bound)
    naive_bytes: int                # sum of all activation tensors (no reuse)
    n_tensors: int
    offsets: List[int] = field(default_factory=list)

    @property
    def per_image_bytes(self) -> float:
        return self.slab_bytes / max(1, self.batch)


def plan_memory(fn: Callable[[], object], batch: int, align: int = 256) -> MemoryPlan:
    """Run ``fn`` once (e.g. ``lambda: model(frames)``) recording every activation
    allocation that goes through :func:`kvedge_amd.ops.empty`, then plan one arena slab
    for them with the native planner.  Lifetimes are in allocation order: a tensor is
    live from its allocation until the allocation that follows its release."""
    sizes: List[int] = []
    first: List[int] = []
    last: List[int] = []
    clock = [0]
    lock = threading.Lock()

    def on_free(i):
        with lock:
            last[i] = clock[0]

    def rec(t: torch.Tensor):
        with lock:
            i = len(sizes)
            sizes.append(t.numel() * t.element_size())
            first.append(clock[0])
            last.append(-1)
            clock[0] += 1
        weakref.finalize(t.untyped_storage(), on_free, i)

    ops.set_alloc_recorder(rec)
    try:
        out = fn()
    finally:
        ops.set_alloc_recorder(None)
    del out
    import gc

    gc.collect()
    end = clock[0]
    last = [end if v < 0 else max(v, f) for v, f in zip(last, first)]
    k = _k()
    if not sizes:
        return MemoryPlan(batch, 0, 0, 0, 0, [])
    res = k.arena_plan(sizes, first, last, align)
    peak = k.arena_live_peak(sizes, first, last)
    return MemoryPlan(batch, int(res[-1]), int(peak), int(sum(sizes)), len(sizes),
                      [int(v) for v in res[:-1]])


def max_batch(plan: MemoryPlan, weight_bytes: int, hbm_bytes: int = HBM_BYTES_MI355X,
              reserve_frac: float = 0.10, frame_bytes_per_image: int = 0) -> int:
    """Largest per-GPU batch whose activations + frames + weights fit in HBM, keeping
    ``reserve_frac`` for the allocator, RCCL buffers and code objects."""
    usable = hbm_bytes * (1.0 - reserve_frac) - weight_bytes
    per = plan.per_image_bytes + frame_bytes_per_image
    return max(0, int(usable // per)) if per > 0 else 0


# ---------------------------------------------------------------------------
# pinned frame ring + native serve loop
# ---------------------------------------------------------------------------
class FrameRing:
    """Pinned host ring of ``slots`` frame batches of ``slot_bytes`` each.

    Producer threads: ``i = ring.acquire_write(timeout_ms)``, fill ``ring.slot(i)``
    (a uint8 CPU tensor view), ``ring.publish(i, seq)``.  The native serve loop drains it.
    """

    def __init__(self, slots: int, slot_bytes: int):
        _k()
        self._r = torch.classes.kvedge.FrameRing(int(slots), int(slot_bytes))

    def acquire_write(self, timeout_ms: int = 1000, drop_oldest: bool = False) -> int:
        return int(self._r.acquire_write(int(timeout_ms), bool(drop_oldest)))

    def slot(self, i: int) -> torch.Tensor:
        return self._r.slot(int(i))

    def publish(self, i: int, seq: int) -> None:
        self._r.publish(int(i), int(seq))

    def put(self, frames: torch.Tensor, seq: int, timeout_ms: int = 1000,
            drop_oldest: bool = False) -> bool:
        """Copy one frame batch (any dtype; bytes must equal slot_bytes) into the ring."""
        i = self.acquire_write(timeout_ms, drop_oldest)
        if i < 0:
            return False
        src = frames.contiguous().view(torch.uint8).reshape(-1)
        self.slot(i).copy_(src)
        self.publish(i, seq)
        return True

    def acquire_read(self, timeout_ms: int = 1000):
        s, seq = self._r.acquire_read(int(timeout_ms))
        return int(s), int(seq)

    def release(self, i: int) -> None:
        self._r.release(int(i))

    def close(self) -> None:
        self._r.close()

    @property
    def dropped(self) -> int:
        return int(self._r.dropped())

    @property
    def ready(self) -> int:
        return int(self._r.ready())

    @property
    def pinned(self) -> bool:
        return bool(self._r.pinned())

    @property
    def slot_bytes(self) -> int:
        return int(self._r.slot_bytes())


@dataclass
class ServeResult:
    steps: int
    wall_s: float
    device_ms: float
    frames_in: int


def serve(graph: "torch.cuda.CUDAGraph", n_steps: int, depth: int = 2,
          hist: Optional[LatencyHistogram] = None, ring: Optional[FrameRing] = None,
          dev_input: Optional[torch.Tensor] = None, ring_timeout_ms: int = 1000,
          device: Optional[int] = None) -> ServeResult:
    """Replay a captured graph ``n_steps`` times from the native loop on torch's current
    stream.  With ``ring``, each step first copies one frame batch into ``dev_input``
    (the graph's fixed input buffer)."""
    k = _k()
    exec_ptr = int(graph.raw_cuda_graph_exec())
    h = hist.data if hist is not None else None
    if ring is not None:
        if dev_input is None:
            raise ValueError("serve(ring=...) needs dev_input, the graph's input buffer")
        r = ring._r.serve(exec_ptr, int(n_steps), int(depth), h, dev_input, int(ring_timeout_ms))
    else:
        dev = torch.cuda.current_device() if device is None else int(device)
        r = k.serve_loop(exec_ptr, int(n_steps), int(depth), h, dev)
    return ServeResult(int(r[0]), float(r[1]), float(r[2]), int(r[3]))
