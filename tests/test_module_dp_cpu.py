"""T-module x T-dist: the edge module with 4 replicas (gloo, one process per rank) stays
in lockstep when events hit only SOME ranks (VERDICT r1 weak #5 / ADVICE high):

  * a ``benchmark`` direct method and a rebuilding ``batch`` twin patch arrive on rank 2
    only, mid-run;
  * a patch that fails to build on rank 3 only (injected) must roll EVERY rank back;
  * the per-rank report clocks disagree (rank r's clock runs r+1 times faster);
  * one rank asks to stop earlier than the others.

Before the control-boundary design any of these hung the job in a collective.  The test
passes if every rank exits, agrees on the final config and rank 2 got its reply.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

WORLD = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, tmp):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch

    torch.set_num_threads(1)
    from kvedge_amd import parallel
    from kvedge_amd.module.app import ModuleApp
    from kvedge_amd.module.config import ModuleConfig
    from kvedge_amd.module.transport import FakeTransport

    class Scripted(FakeTransport):
        """Pushes scripted events into this rank's queue on given poll() calls."""

        def __init__(self, desired, script):
            super().__init__(desired)
            self.script, self.polls = script, 0

        def poll(self):
            self.polls += 1
            for ev in self.script.get(self.polls, []):
                if ev[0] == "twin":
                    self.push_twin_patch(ev[1])
                else:
                    self.invoke_method(ev[1], ev[2])
            super().poll()

    class Clock:  # per-rank clock speeds: report timers disagree across ranks
        def __init__(self):
            self.t = 0.0

        def __call__(self):
            self.t += 0.1 * (rank + 1)
            return self.t

    script = {}
    if rank == 0:  # VM 0's twin is the fleet control point
        script = {3: [("method", "benchmark", {"steps": 1, "warmup": 0}),
                      ("twin", {"batch": 2})],
                  7: [("method", "reconfigure", {"batch": 3})]}
    if rank == 2:  # another device's twin / methods: rejected, never fleet-wide
        script = {3: [("twin", {"batch": 5}), ("method", "reconfigure", {"batch": 6}),
                      ("method", "ping", {})]}
    tr = Scripted({"model": "resnet50", "batch": 1, "image_size": 64,
                   "report_interval_s": 0.5}, script)
    cfg = ModuleConfig(world_size=world, sync_every=2, use_graph=False)
    di = parallel.init_from_env(prefer_gpu=False)
    app = ModuleApp(tr, cfg, device="cpu", state_path=os.path.join(tmp, f"s{rank}.json"),
                    clock=Clock())
    if rank == 3:  # batch 3 cannot be built on rank 3 (e.g. its HBM is exhausted)
        orig = app._build_local

        def failing():
            if app.cfg.batch == 3:
                raise RuntimeError("injected: out of memory")
            orig()

        app._build_local = failing
    try:
        app.start()
        n = app.run(max_steps=10 if rank == 1 else 40)
        app.report()  # final collective report: every rank left run() at one boundary
        res = {n_: (s, r) for n_, s, r in tr.method_results}
        q.put((rank, n, app.cfg.batch, app.boundaries, app.state["rebuilds"],
               app.state["failed_rebuilds"], res, tr.reported.get("lastError", ""),
               len(tr.outputs("telemetry")), di.world_size))
    finally:
        parallel.shutdown()


@pytest.mark.timeout(600)
def test_module_lockstep_4_ranks(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, str(tmp_path)))
             for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=500) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    steps = {r[1] for r in res}
    assert len(steps) == 1, f"ranks left the loop at different steps: {res}"
    n = steps.pop()
    # rank 1 voted to stop at step 10 (boundary 5); the exchange runs with a one-boundary
    # lag, so the fleet applies the vote, and leaves, together at boundary 6
    assert n == 12
    # every rank applied rank 0's batch patch, and rolled back the failing batch=3 together
    assert [r[2] for r in res] == [2] * WORLD
    assert all(r[4] == 2 and r[5] == 1 for r in res)
    assert all(r[3] == n // 2 for r in res)
    r0 = res[0][6]
    assert r0["benchmark"][0] == 200 and r0["benchmark"][1]["world_size"] == WORLD
    assert r0["reconfigure"][0] == 409 and "injected" in r0["reconfigure"][1]["error"]
    assert all("rolled back" in r[7] for r in res if r[0] != 2)
    # rank 2's own twin patch and reconfigure were refused (409), ping still answered
    r2 = res[2][6]
    assert r2["reconfigure"][0] == 409 and "rank 0's twin" in r2["reconfigure"][1]["error"]
    assert r2["ping"][0] == 200
    # only rank 0 emits telemetry (job totals)
    assert res[0][8] >= 1 and all(r[8] == 0 for r in res[1:])


def _module_cmd(tmp, tag):
    import sys

    return [sys.executable, "-m", "kvedge_amd.module", "--transport", "stdout",
            "--model", "resnet50", "--batch", "1", "--image-size", "64", "--no-graph",
            "--steps", "4", "--sync-every", "2", "--report-interval-s", "1000",
            "--state", os.path.join(tmp, f"state-{tag}.json"),
            "--stamps", os.path.join(tmp, f"stamps-{tag}")]


def _telemetry(out):
    import json

    msgs = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
    return [m["payload"] for m in msgs if m.get("output") == "telemetry"]


@pytest.mark.timeout(600)
def test_module_cli_topologies(tmp_path):
    """The chart's per-VM env (kvedge-module-deployment.yaml) drives the module CLI:
    (a) one VM with 2 GPUs -> the module launches 2 local ranks;
    (b) two one-GPU VMs -> two independent processes, KVEDGE_NODE_RANK 0/1."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    base.pop("WORLD_SIZE", None)
    # (a)
    env = dict(base, KVEDGE_NNODES="1", KVEDGE_RANKS_PER_NODE="2", KVEDGE_NODE_RANK="0",
               MASTER_PORT=str(_free_port()))
    r = subprocess.run(_module_cmd(str(tmp_path), "a"), env=env, capture_output=True,
                       text=True, timeout=500, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    tel = _telemetry(r.stdout)
    assert tel and tel[-1]["world_size"] == 2 and {t["rank"] for t in tel} == {0}
    # (b)
    port = str(_free_port())
    procs = [subprocess.Popen(_module_cmd(str(tmp_path), f"b{i}"), cwd=str(tmp_path),
                              env=dict(base, KVEDGE_NNODES="2", KVEDGE_RANKS_PER_NODE="1",
                                       KVEDGE_NODE_RANK=str(i), MASTER_PORT=port),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for i in range(2)]
    outs = [p.communicate(timeout=500) for p in procs]
    assert [p.returncode for p in procs] == [0, 0], outs[1][1][-3000:]
    tel0, tel1 = _telemetry(outs[0][0]), _telemetry(outs[1][0])
    assert tel0 and tel0[-1]["world_size"] == 2 and not tel1
    names = [ln.split()[0] for ln in
             open(os.path.join(str(tmp_path), "stamps-b1")).read().splitlines()]
    assert names[0] == "module_process_start" and names[-1] == "module_first_inference"


def _sync_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    from kvedge_amd import parallel
    from kvedge_amd.module.app import ModuleApp
    from kvedge_amd.module.config import ModuleConfig
    from kvedge_amd.module.transport import FakeTransport

    parallel.init_from_env(prefer_gpu=False)
    tr = FakeTransport({"model": "resnet50", "batch": 1, "image_size": 64,
                        "report_interval_s": 1e9})
    app = ModuleApp(tr, ModuleConfig(world_size=world, sync_every=0, use_graph=False),
                    device="cpu")
    # measured module-step time: 10 ms on rank 0, 50 ms on rank 1 -> rank 0's 20 wins
    app._module_step_s = lambda: 0.010 if rank == 0 else 0.050
    try:
        app.start()
        calls = []
        real_ag = dist.all_gather

        def spy_all_gather(out, t, group=None, async_op=False):
            calls.append((group is parallel.control_group(), async_op, t.device.type))
            return real_ag(out, t, group=group, async_op=async_op)

        def forbidden(*a, **k):
            raise AssertionError("blocking collective on the hot path")

        dist.all_gather = spy_all_gather
        dist.all_reduce = dist.broadcast = dist.all_gather_object = forbidden
        try:
            n = app.run(max_steps=100)
        finally:
            dist.all_gather = real_ag
        q.put((rank, app.sync_every, app.boundaries, n, calls))
    finally:
        parallel.shutdown()


@pytest.mark.timeout(300)
def test_module_auto_sync_every_async_boundaries():
    """boundaries are spaced by measured step time (>= 200 ms: 10 ms
    steps -> every 20 steps, rank 0's measurement adopted by all), and the boundary
    exchange is an ASYNC all_gather on the CPU gloo control group -- no blocking
    collective, nothing on RCCL or a HIP stream, during the serving loop."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sync_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=250) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, sync_every, boundaries, n, calls in res:
        assert sync_every == 20
        # stop voted at step 100 (boundary 5), applied one boundary later
        assert n == 120 and boundaries == 6
        assert len(calls) == boundaries
        assert all(c == (True, True, "cpu") for c in calls), calls
