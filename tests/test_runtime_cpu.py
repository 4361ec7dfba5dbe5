"""Native serving runtime (csrc/runtime) on the CPU tier: latency histogram, arena planner,
pinned frame ring, the C++ self-test and its host-ASan/UBSan build.

The torch bindings are catch-all ops, so the same native code the GPU box runs is tested
here; the serve loop itself needs a GPU (tests/test_runtime_gpu.py)."""
import os
import subprocess
import threading

import numpy as np
import pytest
import torch

from kvedge_amd import ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
needs_lib = pytest.mark.skipif(not ops.load(), reason="kvedge_amd/_C.so not built")


def _hipcc():
    return "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None


@pytest.mark.skipif(_hipcc() is None, reason="hipcc missing")
@pytest.mark.parametrize("asan", [False, True])
def test_native_selftest(tmp_path, asan):
    """Build the C++ self-test (optionally with host ASan + UBSan) and run it."""
    src = [os.path.join(ROOT, "csrc/runtime/selftest_main.cpp"),
           os.path.join(ROOT, "csrc/runtime/kv_runtime.cpp")]
    exe = str(tmp_path / "st")
    cmd = [_hipcc(), "-O1", "-g", "-std=c++17", "--offload-arch=gfx950",
           f"-I{ROOT}/csrc/runtime", *src, "-o", exe]
    if asan:
        cmd[1:1] = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                    "-Xarch_host", "-fno-sanitize-recover=undefined"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK (0 failures)" in r.stdout


@needs_lib
def test_latency_histogram_quantiles_and_merge():
    from kvedge_amd.runtime import LatencyHistogram

    rng = np.random.default_rng(0)
    a_vals = rng.lognormal(mean=8.0, sigma=0.3, size=5000)   # ~3 ms
    b_vals = rng.lognormal(mean=9.0, sigma=0.2, size=3000)   # ~8 ms
    a, b = LatencyHistogram(), LatencyHistogram()
    a.add_many(a_vals)
    for v in b_vals[:10]:
        b.add(v)
    b.add_many(b_vals[10:])
    assert a.count == 5000 and b.count == 3000
    for q in (0.5, 0.9, 0.99):
        exact = np.quantile(a_vals, q)
        assert abs(a.quantiles_us([q])[0] - exact) / exact < 0.035
    allv = np.concatenate([a_vals, b_vals])
    a.merge(b)
    assert a.count == 8000
    assert abs(a.mean_us() - allv.mean()) / allv.mean() < 1e-6
    assert abs(a.percentile_ms(99) - np.quantile(allv, 0.99) / 1e3) / (np.quantile(allv, 0.99) / 1e3) < 0.035
    s = a.summary()
    assert s["p50_ms"] <= s["p90_ms"] <= s["p99_ms"]
    a.reset()
    assert a.count == 0 and a.quantiles_us([0.5]) == [0.0]


@needs_lib
def test_arena_plan_no_live_overlap():
    k = torch.ops.kvedge
    rng = np.random.default_rng(3)
    for _ in range(20):
        n = int(rng.integers(1, 80))
        sizes = [int(v) for v in rng.integers(1, 1 << 20, n)]
        first = [int(v) for v in rng.integers(0, 200, n)]
        last = [f + int(v) for f, v in zip(first, rng.integers(0, 30, n))]
        res = k.arena_plan(sizes, first, last, 256)
        off, total = res[:-1], res[-1]
        assert total >= k.arena_live_peak(sizes, first, last)
        for i in range(n):
            assert off[i] % 256 == 0 and off[i] + sizes[i] <= total
            for j in range(i + 1, n):
                live = first[i] <= last[j] and first[j] <= last[i]
                mem = off[i] < off[j] + sizes[j] and off[j] < off[i] + sizes[i]
                assert not (live and mem)
    with pytest.raises(RuntimeError):
        k.arena_plan([1], [2], [1], 64)


@needs_lib
def test_memory_plan_resnet50_sizes_batch_for_288gb():
    from kvedge_amd import runtime
    from kvedge_amd.engine import InferenceEngine
    from kvedge_amd.models.resnet import KvResNet50

    m = KvResNet50.build(seed=0, device="cpu", calibrate=False)
    eng = InferenceEngine(m, 1, 224, device="cpu")
    plan = eng.memory_plan()
    # two live [56,56,256] bf16 tensors bound the bottleneck stage: 2 * 1.6 MB, plus the
    # input frames / s2d image and the 64-channel intermediates
    big = 56 * 56 * 256 * 2
    assert plan.n_tensors > 50
    assert 2 * big <= plan.slab_bytes <= 4 * big
    assert plan.live_peak_bytes <= plan.slab_bytes < plan.naive_bytes
    wb = sum(t.numel() * t.element_size() for c in m.convs() for t in (c.w, c.b))
    mb = runtime.max_batch(plan, wb, frame_bytes_per_image=224 * 224 * 3)
    assert 10_000 < mb < 200_000  # tens of thousands of images fit in 288 GB


@needs_lib
def test_frame_ring_threads_order_and_drop():
    from kvedge_amd.runtime import FrameRing

    ring = FrameRing(3, 4096)
    assert ring.slot_bytes == 4096
    n = 100
    got = []

    def producer():
        for i in range(n):
            assert ring.put(torch.full((4096,), i % 251, dtype=torch.uint8), i, 5000)

    th = threading.Thread(target=producer)
    th.start()
    while len(got) < n:
        s, seq = ring.acquire_read(5000)
        assert s >= 0
        assert int(ring.slot(s)[4095]) == seq % 251
        got.append(seq)
        ring.release(s)
    th.join()
    assert got == list(range(n))
    r2 = FrameRing(2, 8)
    for i in range(5):
        assert r2.put(torch.zeros(8, dtype=torch.uint8), i, 10, drop_oldest=True)
    assert r2.dropped == 3 and r2.ready == 2
    s, seq = r2.acquire_read(0)
    assert seq == 3
    r2.close()
    assert r2.acquire_write(10) == -1
