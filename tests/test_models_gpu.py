"""T-model: deployed models on the HIP kernels vs the CPU reference path and the fp32 nn.Module."""
import pytest
import torch

from kvedge_amd import ops
from kvedge_amd.engine import InferenceEngine
from kvedge_amd.models.layers import frames_to_nchw
from kvedge_amd.models.resnet import KvResNet50, init_resnet50

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def resnet():
    assert ops.load()
    ref = init_resnet50(seed=0)
    return ref, KvResNet50(ref, "cuda"), KvResNet50(ref, "cpu")


def _frames(n, seed=0, hw=224):
    return torch.randint(0, 256, (n, hw, hw, 3), dtype=torch.uint8,
                         generator=torch.Generator().manual_seed(seed))


def test_resnet50_parity(resnet):
    ref, kv, kv_cpu = resnet
    fr = _frames(3, 1)
    with torch.no_grad():
        lg_gpu = kv.logits(ops.preprocess(fr.cuda())).float().cpu()
        lg_cpu = kv_cpu.logits(ops.preprocess(fr)).float()
        lg_ref = ref(frames_to_nchw(fr)).float()
    cos_dep = torch.nn.functional.cosine_similarity(lg_gpu.flatten(), lg_cpu.flatten(), dim=0)
    cos_ref = torch.nn.functional.cosine_similarity(lg_gpu.flatten(), lg_ref.flatten(), dim=0)
    assert cos_dep > 0.995, float(cos_dep)
    assert cos_ref > 0.98, float(cos_ref)


def test_resnet50_engine_graph(resnet):
    _, kv, _ = resnet
    eng = InferenceEngine(kv, 8, 224, device="cuda", seed=3, use_graph=True).prepare(warmup=1)
    eng.run()
    torch.cuda.synchronize()
    p1 = eng.outputs[0].clone()
    eng.run()
    torch.cuda.synchronize()
    p2 = eng.outputs[0].clone()
    assert torch.isfinite(p1).all()
    assert torch.allclose(p1.sum(1), torch.ones(8, device="cuda"), atol=1e-3)
    # fresh frames every replay -> different outputs
    assert not torch.equal(p1, p2)
    # graph replay == eager on the same frames
    frames = eng.frames.clone()
    probs, _ = kv(frames)
    assert torch.allclose(probs, eng.outputs[0], atol=1e-6)
