"""Scaling-curve runner (kvedge_amd.utils.scaling): the curve math on
synthetic bench lines, and a gloo rehearsal that runs bench.py at N = 1 and 2 (each a
self-launched job) and writes the curve JSON."""
import json

from kvedge_amd.utils import scaling


def _line(n, value, ok=True):
    return {"metric": "m", "unit": "images/sec", "scaling": "weak", "value": value,
            "n_gpus": n, "ms_per_step": 1.0, "dtype": "bf16", "data": "synthetic",
            "config": {"model": "resnet50", "per_gpu_batch": 1280},
            "extra": {"replica_check": {"ok": ok}}}


def test_curve_efficiency_vs_smallest_n():
    c = scaling.curve([_line(4, 380.0), _line(1, 100.0), _line(2, 190.0), _line(8, 720.0)])
    assert c["base_n"] == 1 and c["model"] == "resnet50" and c["scaling"] == "weak"
    assert [p["n_gpus"] for p in c["points"]] == [1, 2, 4, 8]
    assert [p["efficiency"] for p in c["points"]] == [1.0, 0.95, 0.95, 0.9]
    assert c["points"][3]["per_gpu"] == 90.0


def test_scaling_runner_gloo(tmp_path, monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    out = tmp_path / "scaling.json"
    rc = scaling.main(["--cpu", "--gpus", "1,2", "--out", str(out), "--steps", "1",
                       "--warmup", "0"])
    assert rc == 0
    c = json.loads(out.read_text())
    assert [p["n_gpus"] for p in c["points"]] == [1, 2]
    assert all(p["value"] > 0 and p["replica_ok"] for p in c["points"])
    assert c["points"][0]["efficiency"] == 1.0
