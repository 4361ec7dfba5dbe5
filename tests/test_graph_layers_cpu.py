"""tools/graph_layers.py (the round-5 acceptance table) on a synthetic kernel trace: kernels of
two concurrent stream slices are matched back to their layers by stream order, a split-K op
counts its GEMM + finalize launches, and the wall shares add up to the busy time."""
import csv
import io
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tools import graph_layers as gl  # noqa: E402

# per slice: op 0 = one kernel, op 1 = split-K (GEMM + finalize), op 2 = one kernel
NAMES = ["void kvedge::(anonymous namespace)::kA(x)", "kB_gemm", "kB_fin", "kC"]
OP_OF = [0, 1, 1, 2]


def _trace(reps, skew=3000):
    """Two slices; slice 1 starts `skew` ns later, so their kernels overlap.  Durations (ns):
    kA 10000, kB 20000 + fin 5000, kC 4000."""
    dur = [10000, 20000, 5000, 4000]
    rows = [("void kvedge::synth_kernel(...)", 0, 1000)]
    t = 10_000
    for _ in range(reps):
        rows.append(("void kvedge::synth_dev_kernel(...)", t, t + 500))
        for s in range(2):
            ts = t + 1000 + s * skew
            for nm, d in zip(NAMES, dur):
                rows.append((nm, ts, ts + d))
                ts += d + 200
        t += 100_000
    buf = io.StringIO()
    w = csv.writer(buf)
    w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
    for r in rows:
        w.writerow(r)
    return buf.getvalue()


def test_assign_stream_order():
    ks = [(0, 10, "a"), (3, 13, "a"), (11, 30, "b"), (14, 34, "b")]
    out = gl.assign(ks, [0, 1], 2)
    assert out == [(0, 0), (1, 0), (0, 1), (1, 1)]
    # a kernel that starts well before slice 0's previous kernel ended goes to slice 1 even
    # though both slices are at the same op count (stream order)
    ks = [(0, 10000, "a"), (5000, 15000, "a"), (20000, 30000, "b"), (25000, 35000, "b")]
    assert gl.assign(ks, [0, 1], 2) == [(0, 0), (1, 0), (0, 1), (1, 1)]
    # a step whose kernels do not complete every slice's op sequence is refused
    assert gl.assign([(0, 10, "a"), (20, 30, "a"), (40, 50, "c")], [0, 1], 2) is None


def test_summarize_split_k_and_wall_share(tmp_path):
    reps = 3
    trace = tmp_path / "k_kernel_trace.csv"
    trace.write_text(_trace(reps))
    labels = tmp_path / "labels.json"
    labels.write_text(json.dumps({
        "model": "resnet50", "batch": 4, "streams": 2,
        "rows": [["op a", 6e9, 1e12, None], ["op b", 1e9, 1e12, None], ["op c", 1e9, 0.0, None]],
        "kernels": [1, 2, 1]}))
    out = io.StringIO()
    gl.summarize(str(trace), str(labels), reps, 6.0, 2.5, out=out)
    text = out.getvalue()
    table = [ln for ln in text.splitlines() if ln.startswith("| ") and ln[2].isdigit()]
    assert len(table) == 3
    cells = [[c.strip() for c in ln.strip("|").split("|")] for ln in table]
    durs = [float(c[4]) for c in cells]
    # op 1's duration is its GEMM and finalize summed: 25 us; op 0 10 us, op 2 4 us
    assert durs == pytest.approx([10.0, 25.0, 4.0], abs=0.05)
    shares = [float(c[7]) for c in cells]
    busy = float(text.split("GPU busy (union of kernel intervals) ")[1].split(" us")[0])
    other = float(text.split("frames/concat/other kernels: ")[1].split(" us")[0])
    assert sum(shares) + other == pytest.approx(busy, rel=0.01)
    # overlapped layers cost less wall than two full durations
    assert shares[1] < 2 * durs[1]


def test_summarize_refuses_a_short_trace(tmp_path):
    trace = tmp_path / "k_kernel_trace.csv"
    trace.write_text(_trace(1))
    labels = tmp_path / "labels.json"
    labels.write_text(json.dumps({"model": "resnet50", "batch": 4, "streams": 2,
                                  "rows": [["a", 0, 0, None]] * 3, "kernels": [1, 2, 1]}))
    with pytest.raises(SystemExit):
        gl.summarize(str(trace), str(labels), 5, 6.0, 2.5, out=io.StringIO())


def _trace_with_pass(reps):
    """_trace, preceded by the labelled eager pass: bn_kernel before the pass and after every
    op (op 1 = two kernels), plus an earlier unrelated bn_kernel and tuning kernels."""
    pre = [("void kvedge::bn_kernel(...)", -90_000, -89_000), ("kA", -88_000, -87_000)]
    t = -80_000
    seq = [["bn"], ["kA", "bn"], ["kB_gemm", "kB_fin", "bn"], ["kC", "bn"]]
    for grp in seq:
        for nm in grp:
            full = "void kvedge::bn_kernel(...)" if nm == "bn" else nm
            pre.append((full, t, t + 500))
            t += 1000
    body = _trace(reps).splitlines()
    buf = io.StringIO()
    w = csv.writer(buf)
    w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
    for r in pre:
        w.writerow(r)
    return buf.getvalue() + "\n".join(body[1:]) + "\n"


def test_op_kernel_counts_from_separators():
    names = ["bn_kernel", "x", "bn_kernel", "kA", "_ZN6kvedge12_GLOBAL__N_19bn_kernelEPKv", "kB",
             "kB2", "at::native::fill", "kvedge::bn_kernel", "kC", "bn_kernel"]
    assert gl.op_kernel_counts(names, 3) == [1, 2, 1]
    assert gl.op_kernel_counts(names, 11) is None  # no full pass in the trace


def test_summarize_counts_kernels_per_op_from_the_trace(tmp_path):
    """Labels that claim one kernel per op (an op that splits its Cout over two launches, or
    whose kernel count the run step could not know) still summarise: the separator pass in
    the trace gives the real counts."""
    reps = 2
    trace = tmp_path / "k_kernel_trace.csv"
    trace.write_text(_trace_with_pass(reps))
    labels = tmp_path / "labels.json"
    labels.write_text(json.dumps({
        "model": "yolov8n", "batch": 4, "streams": 2,
        "rows": [["op a", 6e9, 1e12, None], ["op b", 1e9, 1e12, None], ["op c", 1e9, 0.0, None]],
        "kernels": [1, 1, 1]}))
    out = io.StringIO()
    gl.summarize(str(trace), str(labels), reps, 6.0, 2.5, out=out)
    table = [ln for ln in out.getvalue().splitlines() if ln.startswith("| ") and ln[2].isdigit()]
    cells = [[c.strip() for c in ln.strip("|").split("|")] for ln in table]
    assert [float(c[4]) for c in cells] == pytest.approx([10.0, 25.0, 4.0], abs=0.05)
    assert "(+1 kernel)" in cells[1][3]
    assert all(float(c[5]) > 0 for c in cells)  # floors come from the op rows
