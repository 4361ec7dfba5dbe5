"""`python -m kvedge_amd.module` -- the IoT Edge module entry point (also bare-metal).

Inside IoT Edge: --transport azure (twin/methods/outputs via edgeHub).  Outside:
--transport stdout prints telemetry as JSON lines; CLI flags mirror the twin keys
 and are overridden by the twin's desired properties.
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import time

from .. import parallel
from .app import GpuUnavailableError, ModuleApp
from .config import ModuleConfig
from .transport import make_transport

_T_IMPORTED = time.time()  # torch, the op library bindings and the module are imported


def _process_start_epoch():
    """Epoch at which the kernel started this process (/proc: boot time + start ticks)."""
    try:
        with open("/proc/self/stat") as f:
            start_ticks = int(f.read().rsplit(")", 1)[1].split()[19])
        with open("/proc/stat") as f:
            btime = next(int(ln.split()[1]) for ln in f if ln.startswith("btime"))
        return btime + start_ticks / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, StopIteration, IndexError):
        return None


def _topology_from_env() -> int:
    """Map the chart's per-VM env (KVEDGE_NODE_RANK / KVEDGE_NNODES /
    KVEDGE_RANKS_PER_NODE, deploy/helm/templates/kvedge-module-deployment.yaml) to
    torch.distributed's.  Returns the number of local ranks this process must launch
    (0 = run in-process)."""
    if "WORLD_SIZE" in os.environ:  # already a launched rank (torchrun / our launcher)
        return 0
    nnodes = int(os.environ.get("KVEDGE_NNODES", "1"))
    rpn = int(os.environ.get("KVEDGE_RANKS_PER_NODE", "1"))
    node = int(os.environ.get("KVEDGE_NODE_RANK", "0"))
    if rpn > 1:
        return rpn
    if nnodes > 1:  # one GPU per VM: this process IS the rank
        os.environ.update(RANK=str(node), LOCAL_RANK="0", WORLD_SIZE=str(nnodes))
    return 0


def main(argv=None):
    local = _topology_from_env()
    if local:
        # topology (a): one VM owns several GPUs -> one child rank per GPU (the parent
        # never touches the GPU); topology (a)+(b) mixes work the same way per VM
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ, PYTHONPATH=os.pathsep.join(
            p for p in (pkg_root, os.environ.get("PYTHONPATH", "")) if p))
        return parallel.launch_local(
            local, ["-m", "kvedge_amd.module", *(sys.argv[1:] if argv is None else argv)],
            env=env,
            node_rank=int(os.environ.get("KVEDGE_NODE_RANK", "0")),
            nnodes=int(os.environ.get("KVEDGE_NNODES", "1")),
            master_addr=os.environ.get("MASTER_ADDR"),
            master_port=int(os.environ["MASTER_PORT"]) if "MASTER_PORT" in os.environ else None)
    d = ModuleConfig()
    ap = argparse.ArgumentParser(prog="kvedge-module")
    ap.add_argument("--transport", default=os.environ.get("KVEDGE_TRANSPORT", "stdout"),
                    choices=["stdout", "fake", "azure"])
    ap.add_argument("--model", default=os.environ.get("KVEDGE_MODEL", d.model))
    ap.add_argument("--batch", type=int, default=int(os.environ.get("KVEDGE_BATCH", d.batch)))
    ap.add_argument("--dtype", default=os.environ.get("KVEDGE_DTYPE", d.dtype))
    ap.add_argument("--seed", type=int, default=d.seed)
    ap.add_argument("--report-interval-s", type=float, default=d.report_interval_s)
    ap.add_argument("--image-size", type=int, default=d.image_size)
    ap.add_argument("--fps", type=float, default=d.fps)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--source", default=d.source, choices=["synthetic", "camera"])
    ap.add_argument("--no-native-loop", action="store_true")
    ap.add_argument("--steps-per-poll", type=int, default=d.steps_per_poll)
    ap.add_argument("--refine-s", type=float, default=d.refine_s,
                    help="seconds of in-graph tile refinement at engine build (0 = off)")
    ap.add_argument("--steps", type=int, default=None, help="stop after N steps")
    ap.add_argument("--duration-s", type=float, default=None)
    ap.add_argument("--sync-every", type=int, default=d.sync_every,
                    help="module steps between lockstep control boundaries (0 = auto)")
    ap.add_argument("--state", default=os.environ.get("KVEDGE_STATE", "/var/lib/kvedge/module-state.json"))
    ap.add_argument("--heartbeat", default=os.environ.get("KVEDGE_HEARTBEAT", ""),
                    help="heartbeat file rewritten at every report (VMI health probes)")
    ap.add_argument("--stamps", default=os.environ.get("KVEDGE_STAMPS", "/var/lib/kvedge/boot-timing"),
                    help="guest boot-timing stamp file (module_first_inference is appended)")
    ap.add_argument("--tune-cache", default=os.environ.get("KVEDGE_TUNE_CACHE",
                                                           "/var/lib/kvedge/tune-cache.json"),
                    help="autotuner picks on the persistent disk ('' = always re-tune)")
    ap.add_argument("--require-gpu", type=int, default=int(os.environ.get("KVEDGE_REQUIRE_GPU", "0") or 0),
                    help="exit non-zero unless at least this many GPUs are visible (the chart "
                         "sets KVEDGE_REQUIRE_GPU from gpu.count; 0 = allow the CPU)")
    a = ap.parse_args(argv)
    di = parallel.init_from_env(prefer_gpu=True)
    cfg = ModuleConfig(model=a.model, batch=a.batch, dtype=a.dtype, seed=a.seed,
                       report_interval_s=a.report_interval_s, image_size=a.image_size,
                       fps=a.fps, use_graph=not a.no_graph, world_size=di.world_size,
                       source=a.source, native_loop=not a.no_native_loop,
                       steps_per_poll=a.steps_per_poll, sync_every=a.sync_every,
                       refine_s=a.refine_s).validate()
    # one IoT Edge identity per VM: only local rank 0 talks to edgeHub
    kind = a.transport if di.local_rank == 0 or a.transport != "azure" else "null"
    try:
        app = ModuleApp(make_transport(kind), cfg, state_path=a.state,
                        stamp_path=a.stamps or None, heartbeat_path=a.heartbeat or None,
                        tune_cache=a.tune_cache or None, require_gpus=a.require_gpu)
    except GpuUnavailableError as e:
        print(str(e), file=sys.stderr, flush=True)
        parallel.shutdown()
        return 3
    # cold-start legs: this process's start (kernel start time) and the end of imports; no
    # process-start stamp when /proc cannot say (a stamp at "now" would corrupt the legs)
    t_start = _process_start_epoch()
    if t_start is not None:
        app._stamp("module_process_start", t_start)
    app._stamp("module_imported", _T_IMPORTED)
    # SIGTERM (edgeAgent stop, VM shutdown) only votes to stop: the replicas leave the
    # loop together at the next control boundary, so the final report's collectives match
    signal.signal(signal.SIGTERM, lambda *_: app.request_stop())
    app.start()
    try:
        app.run(max_steps=a.steps, duration_s=a.duration_s)
        if app.engine is not None:
            app.report()
    finally:
        app.stop()
        parallel.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
