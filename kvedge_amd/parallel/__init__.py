"""N17/N18 data-parallel runtime over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

Inference DP: one replica per GPU (or per one-GPU VM), no
tensor/sequence/expert parallelism — the model fits one MI355X many times over
(25.6 M params = 51 MB bf16 of 288 GB HBM).  Collectives are OFF the per-batch
hot path:
  C1 broadcast of the packed weights from rank 0 once at start (bucketed into
     a few large flat messages: xGMI ring collectives are per-link bound, so
     fewer, larger messages beat many small ones),
  C2 all_reduce(SUM) of throughput counters per report interval,
  C3 all_reduce(MAX) of elapsed time / latency and barriers at phase edges,
  C4 all_gather of output checksums (cross-replica determinism check).
The same code runs on CPU with gloo (tests, world_size > 1 in one container).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Iterable, List, Sequence

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_INFO = DistInfo()


def info() -> DistInfo:
    return _INFO


def init_from_env(prefer_gpu: bool = True) -> DistInfo:
    """Initialise from torchrun env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).

    One process per GPU; backend "nccl" (RCCL) on GPU, "gloo" on CPU.
    """
    global _INFO
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    backend = "none"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if use_gpu else "gloo"
        kw = {"device_id": device} if use_gpu else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    elif dist.is_initialized():
        backend = dist.get_backend()
    _INFO = DistInfo(rank, world, local, backend, device)
    return _INFO


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def barrier():
    if is_dist():
        if _INFO.device.type == "cuda":
            dist.barrier(device_ids=[_INFO.device.index])
        else:
            dist.barrier()


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()


def _flat_buckets(tensors: Sequence[torch.Tensor], bucket_bytes: int):
    """Group same-dtype tensors into buckets of <= bucket_bytes."""
    groups = {}
    for t in tensors:
        groups.setdefault(t.dtype, []).append(t)
    for dtype, ts in groups.items():
        cur, size = [], 0
        for t in ts:
            nb = t.numel() * t.element_size()
            if cur and size + nb > bucket_bytes:
                yield cur
                cur, size = [], 0
            cur.append(t)
            size += nb
        if cur:
            yield cur


def broadcast_tensors(tensors: Sequence[torch.Tensor], src: int = 0,
                      bucket_bytes: int = 64 << 20) -> int:
    """C1: broadcast in-place from ``src`` using large flat buckets.  Returns #messages."""
    if not is_dist():
        return 0
    n = 0
    for bucket in _flat_buckets(list(tensors), bucket_bytes):
        flat = torch.cat([t.reshape(-1) for t in bucket])
        dist.broadcast(flat, src)
        off = 0
        for t in bucket:
            k = t.numel()
            t.copy_(flat[off:off + k].view_as(t))
            off += k
        n += 1
    return n


def allreduce_scalars(vals: Iterable[float], op: str = "sum") -> List[float]:
    """C2/C3: all-reduce a small fp64 vector (counters, elapsed, latency)."""
    v = torch.tensor(list(vals), dtype=torch.float64, device=_INFO.device)
    if is_dist():
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(v, rop)
    return v.cpu().tolist()


def all_gather_scalar(x: float) -> List[float]:
    """C4: gather one float per rank (e.g. an output checksum)."""
    t = torch.tensor([x], dtype=torch.float64, device=_INFO.device)
    if not is_dist():
        return [x]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def model_tensors(model) -> List[torch.Tensor]:
    """All deployed weight/bias tensors of a kvedge model (for C1)."""
    ts = []
    for c in model.convs():
        ts += [c.w, c.b]
    return ts
