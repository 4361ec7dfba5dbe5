"""Multi-stream engine steps (InferenceEngine(streams=S)): the batch is split into S slices,
each run on its own HIP stream as a parallel branch of one hipGraph.  Each slice's outputs
must equal the model run alone on that slice of the same frames (same shapes -> same tiles
-> bitwise), for the graph replay and the eager path, ResNet-50 and YOLOv8n."""
import pytest
import torch

from kvedge_amd import ops
from kvedge_amd.engine import InferenceEngine
from kvedge_amd.models.resnet import KvResNet50, init_resnet50

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kv():
    assert ops.load()
    return KvResNet50(init_resnet50(seed=0), "cuda")


def _per_slice(model, frames, S):
    per = frames.shape[0] // S
    parts = [model(frames[i * per:(i + 1) * per]) for i in range(S)]
    return tuple(torch.cat(xs, 0) for xs in zip(*parts))


@pytest.mark.parametrize("S,graph", [(2, True), (2, False), (4, True)])
def test_resnet_streams_equal_per_slice(kv, S, graph):
    eng = InferenceEngine(kv, 8, 224, device="cuda", seed=7, use_graph=graph,
                          streams=S).prepare(warmup=1, autotune=False)
    for _ in range(3):  # several replays: the frame counter advances inside the graph
        probs, top1 = eng.run()
    torch.cuda.synchronize()
    assert probs.shape == (8, 1000) and top1.shape[0] == 8
    ref_p, ref_t = _per_slice(kv, eng.frames, S)
    torch.cuda.synchronize()
    assert torch.equal(top1, ref_t)
    assert torch.equal(probs, ref_p)


def test_resnet_streams_autotuned_for_slice(kv):
    eng = InferenceEngine(kv, 16, 224, device="cuda", seed=1, streams=2).prepare(warmup=1)
    # the autotuner ran on one 8-image slice: every tuned conv key has batch 8
    assert eng.tuning
    probs, top1 = eng.run()
    torch.cuda.synchronize()
    ref_p, ref_t = _per_slice(kv, eng.frames, 2)
    assert torch.equal(top1, ref_t) and torch.equal(probs, ref_p)


def test_yolo_streams_tuple_outputs():
    from kvedge_amd.models.yolov8 import KvYoloV8n

    y = KvYoloV8n.build(seed=0, device="cuda")
    eng = InferenceEngine(y, 4, 640, device="cuda", seed=2, streams=2).prepare(
        warmup=1, autotune=False)
    out = eng.run()
    torch.cuda.synchronize()
    ref = _per_slice(y, eng.frames, 2)
    assert len(out) == len(ref)
    for a, b in zip(out, ref):
        assert a.shape[0] == 4
        assert torch.equal(a, b)


def test_streams_must_divide_batch(kv):
    with pytest.raises(ValueError):
        InferenceEngine(kv, 6, 224, device="cuda", streams=4)
