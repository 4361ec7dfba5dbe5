"""bench.py's data-parallel contract, rehearsed on the CPU: torchrun with 2 ranks over gloo
runs the same code path the driver launches with N GPUs over RCCL (rendezvous, C1 weight
broadcast, barrier-bracketed timed loop, C3 max-elapsed all-reduce, C4 checksum gather,
one JSON line from rank 0).  `--cpu` swaps the HIP kernels for the reference ops."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world", [2])
def test_bench_dp_contract_gloo(world):
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "1", "--warmup", "0", "--cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    res = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in res, k
    assert res["n_gpus"] == world and res["steps"] == 1 and res["warmup"] == 0
    assert res["scaling"] == "weak" and res["higher_is_better"] is True
    assert res["config"]["parallelism"] == f"dp{world}"
    assert res["config"]["global_batch"] == world * res["config"]["per_gpu_batch"]
    assert res["value"] > 0 and "NOT a measurement" in res["data"]
    assert res["extra"]["backend"] == "gloo"
    rc = res["extra"]["replica_check"]
    assert rc["ok"] and len(rc["digests"]) == world and rc["max_rel_dev"] == 0.0


def _run_bench(args, timeout=900):
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


def test_bench_self_launch_gpus4():
    """No torchrun: ``--gpus 4`` spawns four ranks itself."""
    r = _run_bench(["--cpu", "--gpus", "4", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 4 and res["extra"]["backend"] == "gloo"
    assert res["config"]["parallelism"] == "dp4" and res["config"]["backend"] == "gloo"
    rc = res["extra"]["replica_check"]
    assert rc["ok"] and len(rc["digests"]) == 4
    # all four replicas hashed the same shared-seed frames through identical weights
    assert all(d == rc["digests"][0] for d in rc["digests"])


def test_bench_replica_check_catches_drift():
    """C4 is not vacuous: one rank with perturbed weights fails the run (exit 3)."""
    r = _run_bench(["--cpu", "--gpus", "2", "--steps", "1", "--warmup", "0",
                    "--perturb-rank", "1"])
    assert r.returncode == 3, r.stdout[-2000:] + r.stderr[-4000:]
    assert "replica check FAILED" in r.stderr
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["extra"]["replica_check"]["ok"] is False
    assert res["extra"]["replica_check"]["max_rel_dev"] > 1e-3


def test_bench_rejects_bad_gpus():
    r = _run_bench(["--cpu", "--gpus", "0"], timeout=300)
    assert r.returncode == 2 and "--gpus must be" in r.stderr


def test_bench_refuses_more_gpus_than_visible():
    r = _run_bench(["--gpus", "2"], timeout=300)  # no --cpu; this host sees 0 GPUs
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr


def _ranks_alive(marker: str):
    import psutil

    out = []
    for p in psutil.process_iter(["pid", "cmdline"]):
        cl = p.info.get("cmdline") or []
        if any("bench.py" in c for c in cl) and marker in cl:
            out.append(p)
    return out


def test_bench_launcher_timeout_kills_hung_rank():
    """a rank that never arrives (hung RCCL init) must not hang the
    job.  --launch-timeout bounds it: non-zero exit, every rank gone, stderr prefixed."""
    import time

    marker = "424242"  # unique --seed value to find our own ranks afterwards
    t0 = time.monotonic()
    r = _run_bench(["--cpu", "--gpus", "2", "--steps", "1", "--warmup", "0", "--seed", marker,
                    "--hang-rank", "1", "--launch-timeout", "15"], timeout=120)
    assert r.returncode == 124, r.stderr[-3000:]
    assert time.monotonic() - t0 < 60
    assert "[launcher] timeout" in r.stderr
    assert not _ranks_alive(marker)


def test_bench_launcher_forwards_sigterm():
    """SIGTERM to the launcher (driver / edgeAgent stop) reaches every rank; nothing
    survives the grace period."""
    import signal
    import time

    marker = "434343"
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2",
                          "--steps", "1", "--warmup", "0", "--seed", marker, "--hang-rank", "1"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, cwd=ROOT)
    try:
        deadline = time.monotonic() + 60
        while len(_ranks_alive(marker)) < 3 and time.monotonic() < deadline:
            time.sleep(0.2)  # launcher + 2 ranks
        assert len(_ranks_alive(marker)) == 3
        p.send_signal(signal.SIGTERM)
        _, err = p.communicate(timeout=40)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode != 0
    assert b"[launcher] signal 15" in err
    time.sleep(0.5)
    assert not _ranks_alive(marker)


def test_launcher_peer_failure_is_bounded(tmp_path):
    """One rank dies; its peer is stuck in a collective.  The launcher SIGTERMs it and
    escalates to SIGKILL after the grace period instead of waiting for the gloo/RCCL
    timeout; each rank's stderr carries its rank prefix."""
    import time

    from kvedge_amd import parallel

    script = tmp_path / "rank.py"
    script.write_text(
        "import os, signal, sys, time\n"
        "r = int(os.environ['RANK'])\n"
        "print('hello from', r, file=sys.stderr, flush=True)\n"
        "if r == 1:\n"
        "    time.sleep(0.5); sys.exit(7)\n"
        "signal.signal(signal.SIGTERM, signal.SIG_IGN)  # a rank that ignores SIGTERM\n"
        "time.sleep(600)\n")
    import io
    import contextlib

    buf = io.BytesIO()

    class _Err:
        buffer = buf

        def write(self, s):
            buf.write(s.encode())

        def flush(self):
            pass

    t0 = time.monotonic()
    with contextlib.redirect_stderr(_Err()):
        rc = parallel.launch_local(2, [str(script)], grace_s=2.0)
    assert rc == 7
    assert time.monotonic() - t0 < 20
    txt = buf.getvalue().decode()
    assert "[rank 0] hello from 0" in txt and "[rank 1] hello from 1" in txt
