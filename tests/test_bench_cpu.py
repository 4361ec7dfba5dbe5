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
