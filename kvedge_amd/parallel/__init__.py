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
from typing import Iterable, List, Optional, Sequence

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


def launch_local(nproc: int, argv: Sequence[str], env: Optional[dict] = None,
                 timeout_s: Optional[float] = None, node_rank: int = 0, nnodes: int = 1,
                 master_addr: Optional[str] = None, master_port: Optional[int] = None) -> int:
    """Per-node launcher (the torchrun role, without its agent): start ``nproc``
    fresh child processes ``python <argv>`` with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set,
    one per GPU, wait for all, return the first non-zero exit code (0 if all passed).
    Multi-node (e.g. several 8-GPU VMs): global rank = node_rank * nproc + local rank,
    and every node must be given the same master_addr/port (rank 0's node).

    The parent must not have touched the GPU (a process that initialised HIP must not
    be replaced or fork GPU children); it only counts devices.  If one rank fails, the
    others would block in their next collective, so the survivors are terminated.
    """
    import socket
    import subprocess
    import sys
    import time

    if master_port is None:
        if nnodes > 1:
            raise ValueError("multi-node launch needs an explicit master_port")
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        master_port = s.getsockname()[1]
        s.close()
    addr = master_addr or "127.0.0.1"
    base = dict(os.environ if env is None else env)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host
    procs = []
    for r in range(nproc):
        e = dict(base, RANK=str(node_rank * nproc + r), LOCAL_RANK=str(r),
                 WORLD_SIZE=str(nnodes * nproc), LOCAL_WORLD_SIZE=str(nproc),
                 MASTER_ADDR=addr, MASTER_PORT=str(master_port))
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    rc = 0
    t_end = None if timeout_s is None else time.monotonic() + timeout_s
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # peers would hang in their next collective
                    q.terminate()
        if t_end is not None and time.monotonic() > t_end:
            for q in pending:
                q.kill()
            rc = rc or 124
            break
        time.sleep(0.05)
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc if rc >= 0 else 128 - rc


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


def all_gather_vector(vals: Sequence[float]) -> List[List[float]]:
    """C4: gather a small fp64 vector per rank -> [world][len(vals)]."""
    t = torch.tensor(list(vals), dtype=torch.float64, device=_INFO.device)
    if not is_dist():
        return [t.cpu().tolist()]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def all_gather_object(obj) -> list:
    """Gather one small picklable control object per rank (module lockstep boundary:
    queued twin patches / method calls, stop flags).  Identity at world size 1."""
    if not is_dist():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def digest(t: torch.Tensor) -> List[float]:
    """Order-sensitive fp64 digest of a tensor: [sum, sum of squares, position-weighted
    sum].  The weights (1 + i mod 97) make a permutation or a sign flip visible, which a
    plain sum (e.g. of softmax probabilities, always == batch) cannot see."""
    x = t.detach().reshape(-1).double()
    w = (torch.arange(x.numel(), device=x.device, dtype=torch.float64) % 97) + 1.0
    return [float(x.sum()), float((x * x).sum()), float((x * w).sum())]


@dataclass
class ReplicaCheck:
    ok: bool
    max_rel_dev: float
    digests: List[List[float]]


def check_replicas(local: Sequence[float], rtol: float = 1e-4) -> ReplicaCheck:
    """C4 cross-replica determinism: every rank computed ``local`` (a :func:`digest`) on
    the SAME input with its own copy of the weights and kernels; all ranks must agree
    with rank 0 within ``rtol`` (relative to rank 0's magnitude per component).  Same
    kernels and the same (fleet-autotuned) tiles on identical hardware are bitwise
    deterministic, so a deviation means a replica drifted (weights, tile, fault)."""
    rows = all_gather_vector(local)
    ref = rows[0]
    dev = 0.0
    for r in rows[1:]:
        for a, b in zip(r, ref):
            dev = max(dev, abs(a - b) / max(abs(b), 1e-30))
    finite = all(x == x and abs(x) != float("inf") for r in rows for x in r)
    return ReplicaCheck(finite and dev <= rtol, dev, rows)


def model_tensors(model) -> List[torch.Tensor]:
    """All deployed weight/bias tensors of a kvedge model (for C1)."""
    ts = []
    for c in model.convs():
        ts += [c.w, c.b]
    return ts
