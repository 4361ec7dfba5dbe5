"""tools/bench_line.py (the same-box A/B scripts' one-line summary of a bench.py JSON line): the
headline, every edge batch and the YOLOv8n extra are reported; a run without extras still
prints the headline."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, doc):
    f = tmp_path / "b.txt"
    f.write_text("some log line\n" + json.dumps(doc) + "\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_line.py"), str(f)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


def test_bench_line_full(tmp_path):
    doc = {"value": 88778.4, "ms_per_step": 14.418,
           "extra": {"edge": [{"batch": 1, "p50_ms": 0.2774, "images_per_s": 3605.0},
                              {"batch": 64, "p50_ms": 1.1312, "images_per_s": 56578.0}],
                     "yolov8n": {"value": 55081.2}}}
    out = _run(tmp_path, doc)
    assert out.startswith("headline 88778 (14.418 ms)")
    assert "b1 0.2774 ms 3605/s" in out and "b64 1.1312 ms 56578/s" in out
    assert out.endswith("yolo 55081")


def test_bench_line_headline_only(tmp_path):
    assert _run(tmp_path, {"value": 53846.0, "ms_per_step": 9.508}) == "headline 53846 (9.508 ms)"
