"""Native serving runtime on the MI355X: the C++ serve loop replaying the engine's hipGraph,
fed either by on-device synthetic frames or by the pinned FrameRing (real-frame ingest)."""
import os
import subprocess
import threading

import pytest
import torch

from kvedge_amd import ops
from kvedge_amd.engine import InferenceEngine
from kvedge_amd.models.resnet import KvResNet50, init_resnet50

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def kv():
    assert ops.load()
    return KvResNet50(init_resnet50(seed=0), "cuda")


def test_native_selftest_binary_on_gpu():
    exe = os.path.join(ROOT, "kvedge_amd", "bin", "kv_runtime_selftest")
    assert os.path.exists(exe), "build with python -m kvedge_amd._build"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "serve_loop: 32 steps" in r.stdout


def test_serve_native_matches_python_replay(kv):
    from kvedge_amd.runtime import LatencyHistogram

    a = InferenceEngine(kv, 8, 224, device="cuda", seed=5).prepare(warmup=1, autotune=False)
    b = InferenceEngine(kv, 8, 224, device="cuda", seed=5).prepare(warmup=1, autotune=False)
    # same number of steps from the same counter state -> same synthetic frames
    a.step_ctr.zero_()
    b.step_ctr.zero_()
    for _ in range(6):
        a.run()
    h = LatencyHistogram()
    res = b.serve_native(6, depth=3, hist=h)
    torch.cuda.synchronize()
    assert res.steps == 6 and h.count == 6
    assert res.device_ms > 0 and h.percentile_ms(50) > 0
    assert torch.equal(a.outputs[1], b.outputs[1])
    assert torch.allclose(a.outputs[0], b.outputs[0])


def test_ring_fed_serving_equals_set_frames(kv):
    from kvedge_amd.runtime import FrameRing, LatencyHistogram

    B = 4
    frames = [torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8,
                            generator=torch.Generator().manual_seed(i)) for i in range(3)]
    eng = InferenceEngine(kv, B, 224, device="cuda", synthetic=False).prepare(
        warmup=1, autotune=False)
    ring = FrameRing(2, eng.frames.numel())
    assert ring.pinned

    def producer():
        for i, f in enumerate(frames):
            assert ring.put(f, i, timeout_ms=10_000)

    th = threading.Thread(target=producer)
    th.start()
    h = LatencyHistogram()
    res = eng.serve_native(3, depth=2, hist=h, ring=ring, ring_timeout_ms=10_000)
    th.join()
    torch.cuda.synchronize()
    assert res.frames_in == 3 and h.count == 3
    probs_ring = eng.outputs[0].clone()
    # the same last batch through the eager path
    ref = InferenceEngine(kv, B, 224, device="cuda", use_graph=False, synthetic=False)
    out = ref.set_frames(frames[-1].cuda())
    torch.cuda.synchronize()
    # the ring delivered exactly the last batch: identical frames -> identical logits
    assert torch.equal(eng.frames.cpu(), frames[-1])
    with torch.no_grad():
        lg_ring = kv.raw_outputs(eng.frames).float()
        lg_ref = kv.raw_outputs(frames[-1].cuda()).float()
    assert torch.equal(lg_ring, lg_ref)
    assert torch.allclose(probs_ring, out[0], rtol=1e-3, atol=1e-7)
    assert torch.equal(probs_ring.argmax(1), torch.softmax(lg_ref, 1).argmax(1))
    ring.close()


@pytest.mark.parametrize("source", ["camera", "synthetic"])
def test_module_native_serving(source):
    """The edge module on the GPU: native serve loop (4 graph replays per poll), fed by the
    camera thread through the pinned ring or by the on-device generator."""
    from kvedge_amd.module.app import ModuleApp
    from kvedge_amd.module.transport import FakeTransport

    tr = FakeTransport({"model": "resnet50", "batch": 8, "report_interval_s": 0.01,
                        "source": source, "steps_per_poll": 4})
    # a failed assertion must still stop the camera thread (a daemon thread left in the
    # native ring.put() at interpreter exit is std::terminate): context manager
    with ModuleApp(tr, device="cuda").start() as app:
        assert app.engine.graph is not None
        app.run(max_steps=3)
        app.report()  # may follow an auto-report: then it carries that window
        t = tr.outputs("telemetry")[-1]
        assert t["source"] == source and t["images_per_s"] > 0
        assert app.state["total_images"] == 3 * 4 * 8
        if source == "camera":
            assert app.ring.pinned and app.camera.seq >= 12
