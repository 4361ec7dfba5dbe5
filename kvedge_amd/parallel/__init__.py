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


# Child bootstrap of launch_local, run as ``python -c _RANK_BOOT <argv...>``.  It arms
# PR_SET_PDEATHSIG in the (single-threaded, GPU-clean) child itself, so the launcher
# needs no ``preexec_fn``: that hook runs Python in the forked child while the parent's
# stderr pump threads may hold the allocator or loader locks, and it
# forces a fork+exec instead of posix_spawn.  If the launcher died before the signal
# was armed, the child's parent is no longer the launcher: exit at once.
_RANK_BOOT = r"""
import ctypes, os, runpy, signal, sys
try:
    ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGTERM))  # PR_SET_PDEATHSIG
except (OSError, AttributeError):
    pass
if os.getppid() != int(os.environ.get("KVEDGE_LAUNCHER_PID", os.getppid())):
    sys.exit(143)
args = sys.argv[1:]
if args[:1] == ["-m"]:
    sys.argv = [args[1]] + args[2:]
    runpy.run_module(args[1], run_name="__main__", alter_sys=True)
else:
    sys.argv = list(args)
    sys.path.insert(0, os.path.dirname(os.path.abspath(args[0])))
    runpy.run_path(args[0], run_name="__main__")
"""


_KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def visible_gpu_count(topology: Optional[str] = None) -> int:
    """Number of GPUs this process would see, WITHOUT initialising HIP.

    ``torch.cuda.device_count()`` on ROCm falls back to ``hipGetDeviceCount`` when amdsmi
    is unavailable, which initialises the HIP runtime in the caller; a launcher that then
    forks GPU ranks breaks the rule that a GPU-initialised process never spawns or execs
    GPU work.  This reads the KFD topology instead: one node per agent, GPUs are the nodes
    whose ``gfx_target_version`` is non-zero (CPU nodes report 0).  The visibility masks
    are applied in the runtime's order: ROCR_VISIBLE_DEVICES selects among the agents,
    then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES index into what is left.
    The sysfs topology is not per-container: a process that a cgroup / device plugin
    limits to some of the render nodes still sees every GPU there.  Like the ROCm runtime,
    which enumerates only the agents whose ``/dev/dri/renderD<drm_render_minor>`` it can
    open, a GPU node counts only if that node is readable and writable.
    ``KVEDGE_KFD_TOPOLOGY`` / ``KVEDGE_DRI_ROOT`` override the sysfs and /dev/dri roots
    (tests)."""
    import glob

    root = topology or os.environ.get("KVEDGE_KFD_TOPOLOGY", _KFD_TOPOLOGY)
    dri = os.environ.get("KVEDGE_DRI_ROOT", "/dev/dri")
    check_dri = os.path.isdir(dri)  # no /dev/dri view at all: nothing to check against
    n = 0
    for prop in sorted(glob.glob(os.path.join(root, "*", "properties"))):
        try:
            kv = {}
            with open(prop) as f:
                for ln in f:
                    k, _, v = ln.partition(" ")
                    kv[k] = v.strip()
            if int(kv.get("gfx_target_version", "0") or 0) == 0:
                continue
            minor = kv.get("drm_render_minor")
            if check_dri and minor is not None and int(minor) > 0:
                node = os.path.join(dri, f"renderD{int(minor)}")
                if not os.access(node, os.R_OK | os.W_OK):
                    continue  # masked from this container / cgroup
            n += 1
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        mask = os.environ.get(var)
        if mask is None:
            continue
        ids = [x.strip() for x in mask.split(",") if x.strip()]
        valid = []
        for x in ids:
            if x.isdigit() and int(x) < n:
                valid.append(x)
            elif not x.isdigit() and x.upper().startswith("GPU-"):
                valid.append(x)  # UUID form: cannot be checked without HIP, trust it
            else:
                break  # the runtime stops at the first invalid entry
        n = len(valid)
    return n


def _pump_prefixed(stream, out, prefix: bytes):
    """Copy a rank's stderr line by line, each line prefixed with its rank."""
    try:
        for line in iter(stream.readline, b""):
            out.write(prefix + line)
            out.flush()
    except (OSError, ValueError):
        pass
    finally:
        stream.close()


def launch_local(nproc: int, argv: Sequence[str], env: Optional[dict] = None,
                 timeout_s: Optional[float] = None, node_rank: int = 0, nnodes: int = 1,
                 master_addr: Optional[str] = None, master_port: Optional[int] = None,
                 grace_s: float = 10.0, prefix_stderr: bool = True) -> int:
    """Per-node launcher (the torchrun role, without its agent): start ``nproc``
    fresh child processes ``python <argv>`` with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set,
    one per GPU, wait for all, return the first non-zero exit code (0 if all passed).
    Multi-node (e.g. several 8-GPU VMs): global rank = node_rank * nproc + local rank,
    and every node must be given the same master_addr/port (rank 0's node).

    The parent must not have touched the GPU (a process that initialised HIP must not
    be replaced or fork GPU children); it counts devices with :func:`visible_gpu_count`
    (sysfs, no HIP).  Children are spawned without a ``preexec_fn`` and arm their own
    parent-death signal (``_RANK_BOOT``).

    Stop paths, all bounded:
      * one rank exits non-zero -> its peers would block in their next collective until
        the RCCL timeout, so they get SIGTERM, then SIGKILL after ``grace_s``;
      * SIGTERM / SIGINT to the launcher (edgeAgent stop: the launcher is the module
        container's PID 1) -> forwarded to every rank (the module turns it into a fleet
        stop vote and writes its final report + state file), SIGKILL after ``grace_s``;
      * ``timeout_s`` -> every rank is SIGTERMed, then SIGKILLed; exit code 124;
      * the launcher itself SIGKILLed -> the kernel SIGTERMs the ranks (PDEATHSIG).
    Each rank's stderr is prefixed ``[rank R] ``; stdout passes through unchanged (the
    bench's one JSON line).
    """
    import signal
    import socket
    import subprocess
    import sys
    import threading
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
    base.setdefault("PYTHONUNBUFFERED", "1")  # prefixed stderr lines arrive as written
    base["KVEDGE_LAUNCHER_PID"] = str(os.getpid())
    procs, pumps = [], []
    got_signal = []

    def _on_signal(signum, _frame):
        got_signal.append(signum)

    main_thread = threading.current_thread() is threading.main_thread()
    old = {}
    if main_thread:
        for sig in (signal.SIGTERM, signal.SIGINT):
            old[sig] = signal.signal(sig, _on_signal)
    try:
        for r in range(nproc):
            grank = node_rank * nproc + r
            e = dict(base, RANK=str(grank), LOCAL_RANK=str(r),
                     WORLD_SIZE=str(nnodes * nproc), LOCAL_WORLD_SIZE=str(nproc),
                     MASTER_ADDR=addr, MASTER_PORT=str(master_port))
            p = subprocess.Popen([sys.executable, "-c", _RANK_BOOT] + list(argv), env=e,
                                 stderr=subprocess.PIPE if prefix_stderr else None)
            procs.append(p)
        if prefix_stderr:  # pumps start only once every rank is spawned
            for r, p in enumerate(procs):
                t = threading.Thread(target=_pump_prefixed, daemon=True,
                                     args=(p.stderr, sys.stderr.buffer,
                                           f"[rank {node_rank * nproc + r}] ".encode()))
                t.start()
                pumps.append(t)
        rc = 0
        t_end = None if timeout_s is None else time.monotonic() + timeout_s
        kill_at = None  # SIGKILL deadline once the survivors were asked to stop
        pending = list(procs)

        def _stop_all(why: str):
            nonlocal kill_at
            if kill_at is None:
                print(f"[launcher] {why}: stopping {len(pending)} rank(s) "
                      f"(SIGTERM, SIGKILL after {grace_s:g} s)", file=sys.stderr, flush=True)
                for q in pending:
                    try:
                        q.send_signal(signal.SIGTERM)
                    except OSError:
                        pass
                kill_at = time.monotonic() + grace_s

        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    if pending:
                        _stop_all(f"rank {procs.index(p) + node_rank * nproc} exited {code}")
            if got_signal and kill_at is None:  # rc stays the ranks' own exit codes
                _stop_all(f"signal {got_signal[0]}")
            if t_end is not None and time.monotonic() > t_end and kill_at is None:
                rc = rc or 124
                _stop_all(f"timeout after {timeout_s:g} s")
            if kill_at is not None and time.monotonic() > kill_at:
                for q in pending:
                    q.kill()
                for q in pending:
                    q.wait()
                pending = []
                break
            time.sleep(0.05)
        for p in procs:
            try:
                p.wait(timeout=grace_s)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for t in pumps:
            t.join(timeout=2)
    finally:
        for p in procs:  # never leave a rank behind, whatever happened above
            if p.poll() is None:
                p.kill()
                p.wait()
        for sig, h in old.items():
            signal.signal(sig, h)
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


def all_gather_object(obj, group=None) -> list:
    """Gather one small picklable control object per rank (build-time agreement: desired
    config, build errors, the auto sync interval).  Identity at world size 1.  Pass
    ``group=control_group()`` to keep it on the CPU gloo group (no HIP stream, no RCCL)."""
    if not is_dist():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj, group=group)
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


_CTL_GROUP = None


def control_group():
    """CPU (gloo) process group for the module's control plane: lockstep boundary
    exchanges never touch RCCL or a HIP stream, so they cannot queue behind (or in
    front of) inference work on the device.  Collective: every rank must call it the
    first time.  None at world size 1."""
    global _CTL_GROUP
    if not is_dist():
        return None
    if _CTL_GROUP is None:
        _CTL_GROUP = dist.new_group(backend="gloo")
    return _CTL_GROUP


class ObjectExchange:
    """Asynchronous all-gather of one small picklable object per rank over the gloo
    control group (module lockstep boundary, SURVEY §2.6: collectives off the hot path).

    ``post(obj)`` serialises into a fixed ``capacity``-byte slot and starts a
    non-blocking all_gather; ``wait()`` returns the per-rank objects.  The module posts
    at boundary k and waits at boundary k+1, so the exchange overlaps a whole boundary
    interval of inference instead of stalling the step that reaches the boundary.
    """

    HEADER = 8

    def __init__(self, capacity: int = 64 << 10, group=None):
        self.capacity = capacity
        self.group = group if group is not None else control_group()
        self.world = dist.get_world_size() if is_dist() else 1
        self._work = None
        self._out = None
        self.posted = 0

    @property
    def pending(self) -> bool:
        return self._work is not None or self._out is not None

    def fits(self, obj) -> bool:
        import pickle

        return len(pickle.dumps(obj, protocol=4)) <= self.capacity - self.HEADER

    def post(self, obj) -> None:
        import pickle

        if self.pending:
            raise RuntimeError("ObjectExchange: previous exchange not collected")
        raw = pickle.dumps(obj, protocol=4)
        if len(raw) > self.capacity - self.HEADER:
            raise ValueError(f"control payload {len(raw)} B exceeds {self.capacity} B")
        buf = torch.zeros(self.capacity, dtype=torch.uint8)
        buf[:self.HEADER] = torch.tensor(list(len(raw).to_bytes(self.HEADER, "little")),
                                         dtype=torch.uint8)
        buf[self.HEADER:self.HEADER + len(raw)] = torch.frombuffer(bytearray(raw),
                                                                   dtype=torch.uint8)
        self.posted += 1
        if self.world == 1:
            self._out = [buf]
            return
        self._out = [torch.empty_like(buf) for _ in range(self.world)]
        self._work = dist.all_gather(self._out, buf, group=self.group, async_op=True)

    def wait(self) -> list:
        import pickle

        if not self.pending:
            raise RuntimeError("ObjectExchange: nothing posted")
        if self._work is not None:
            self._work.wait()
        out, self._work, self._out = self._out, None, None
        res = []
        for b in out:
            n = int.from_bytes(bytes(b[:self.HEADER].tolist()), "little")
            res.append(pickle.loads(b[self.HEADER:self.HEADER + n].numpy().tobytes()))
        return res
