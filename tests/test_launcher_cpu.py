"""The N-GPU launchers must stay GPU-clean.

``bench.py --gpus N`` and ``python -m kvedge_amd.utils.scaling`` are the parents of the GPU
ranks.  On this pool a process that has initialised HIP must never fork or exec GPU work,
and on ROCm ``torch.cuda.device_count()`` can initialise HIP (hipGetDeviceCount when amdsmi
is missing).  These tests run both launchers with every torch.cuda entry point that could
touch HIP replaced by a function that raises, and check devices are counted from sysfs."""
import json
import os
import subprocess
import sys

import pytest

from kvedge_amd import parallel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# run a launcher in a fresh interpreter whose torch.cuda cannot be touched
_POISON = r"""
import runpy, sys
import torch

def _boom(*a, **k):
    raise AssertionError("launcher touched HIP via torch.cuda")

torch.cuda.device_count = _boom
torch.cuda.is_available = _boom
torch.cuda.init = _boom
torch.cuda.set_device = _boom
torch._C._cuda_getDeviceCount = _boom
target, args = sys.argv[1], sys.argv[2:]
if target.endswith(".py"):
    sys.argv = [target] + args
    runpy.run_path(target, run_name="__main__")
else:
    sys.argv = [target] + args
    runpy.run_module(target, run_name="__main__", alter_sys=True)
"""


def _fake_topology(root, gfx_versions):
    for i, v in enumerate(gfx_versions):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if v else 8}\n"
                                      f"simd_count {1024 if v else 0}\n"
                                      f"gfx_target_version {v}\n")
    return str(root)


def _env(**kw):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        env.pop(k, None)
    env.update(kw)
    return env


def _poisoned(target, args, env, timeout=900):
    return subprocess.run([sys.executable, "-c", _POISON, target] + list(args),
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


def test_visible_gpu_count_from_sysfs(tmp_path, monkeypatch):
    topo = _fake_topology(tmp_path / "nodes", [0, 0, 90500, 90500, 90500])  # 2 CPUs, 3 GPUs
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    assert parallel.visible_gpu_count(topo) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,0")
    assert parallel.visible_gpu_count(topo) == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")  # ROCR first: 1 agent left ...
    assert parallel.visible_gpu_count(topo) == 0  # ... so HIP index 2 is invalid
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert parallel.visible_gpu_count(topo) == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert parallel.visible_gpu_count(topo) == 0
    assert parallel.visible_gpu_count(str(tmp_path / "missing")) == 0


def test_visible_gpu_count_skips_masked_render_nodes(tmp_path, monkeypatch):
    """sysfs lists every GPU of the host; a container limited to some
    render nodes must count only the GPUs whose /dev/dri/renderD<minor> it can open."""
    topo = _fake_topology(tmp_path / "nodes", [0, 90500, 90500, 90500])
    for i, minor in ((1, 128), (2, 129), (3, 130)):
        with open(tmp_path / "nodes" / str(i) / "properties", "a") as f:
            f.write(f"drm_render_minor {minor}\n")
    dri = tmp_path / "dri"
    dri.mkdir()
    for minor in (128, 130):
        (dri / f"renderD{minor}").write_text("")
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("KVEDGE_DRI_ROOT", str(dri))
    assert parallel.visible_gpu_count(topo) == 2
    (dri / "renderD129").write_text("")
    assert parallel.visible_gpu_count(topo) == 3
    monkeypatch.setenv("KVEDGE_DRI_ROOT", str(tmp_path / "no-dri"))  # no view: trust sysfs
    assert parallel.visible_gpu_count(topo) == 3


def test_bench_launcher_never_touches_hip(tmp_path):
    """GPU path of the launcher: devices counted from sysfs; too few -> clean refusal,
    and no torch.cuda call on the way."""
    topo = _fake_topology(tmp_path / "nodes", [0, 90500])
    r = _poisoned(os.path.join(ROOT, "bench.py"), ["--gpus", "2"],
                  _env(KVEDGE_KFD_TOPOLOGY=topo), timeout=300)
    assert r.returncode == 2, r.stdout[-2000:] + r.stderr[-4000:]
    assert "only 1 GPU(s) visible" in r.stderr and "touched HIP" not in r.stderr


def test_bench_cpu_self_launch_with_poisoned_cuda():
    """--cpu --gpus 2 launches and passes with torch.cuda poisoned in the parent."""
    r = _poisoned(os.path.join(ROOT, "bench.py"),
                  ["--cpu", "--gpus", "2", "--steps", "1", "--warmup", "0"],
                  _env(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    res = json.loads(lines[-1])
    assert res["n_gpus"] == 2 and res["extra"]["replica_check"]["ok"]


def test_scaling_launcher_never_touches_hip(tmp_path):
    topo = _fake_topology(tmp_path / "nodes", [0])  # no GPU at all
    r = _poisoned("kvedge_amd.utils.scaling", ["--gpus", "1,2"],
                  _env(KVEDGE_KFD_TOPOLOGY=topo), timeout=300)
    assert r.returncode == 2 and "no runnable GPU counts" in r.stderr, r.stderr[-3000:]
    assert "touched HIP" not in r.stderr


@pytest.mark.parametrize("ns", ["1,2"])
def test_scaling_cpu_with_poisoned_cuda(tmp_path, ns):
    out = tmp_path / "curve.json"
    r = _poisoned("kvedge_amd.utils.scaling",
                  ["--cpu", "--gpus", ns, "--out", str(out), "--steps", "1", "--warmup", "0"],
                  _env(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    c = json.loads(out.read_text())
    assert [p["n_gpus"] for p in c["points"]] == [1, 2]


def test_launcher_children_have_parent_death_signal(tmp_path):
    """Children arm PR_SET_PDEATHSIG themselves (no preexec_fn in the launcher)."""
    script = tmp_path / "rank.py"
    script.write_text(
        "import ctypes, os, sys\n"
        "sig = ctypes.c_int(0)\n"
        "ctypes.CDLL(None).prctl(2, ctypes.byref(sig))  # PR_GET_PDEATHSIG\n"
        "assert sig.value == 15, sig.value\n"
        "assert sys.argv[1:] == ['--x', '1'], sys.argv\n"
        "assert os.environ['KVEDGE_LAUNCHER_PID'] == str(os.getppid())\n")
    assert parallel.launch_local(2, [str(script), "--x", "1"], grace_s=2.0,
                                 prefix_stderr=False) == 0
