"""The edge-serving configurations: ResNet-50 at the module's
batch sizes (b1 / b8 / b64; twin default 64, deploy/helm/values.yaml module.batch) as
`edge_latency` and the module serve them -- per-batch autotuned tiles (split-K forms at
small M, their per-stream fp32 slab workspace shared by every split-K layer), one hipGraph
-- checked against the fp32 nn.Module on the frames the graph itself synthesised.

Between capture and replay every split-K workspace is poisoned with NaN: no output may
depend on what an earlier layer (or an earlier replay) left in a slab.  The fused edge head
(ops.pooled_fc, avgpool + fc in one launch) is checked against the unfused head at the
model level for B in {1, 16}."""
import copy

import pytest
import torch

from kvedge_amd import ops
from kvedge_amd.engine import InferenceEngine, edge_streams

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def models():
    from kvedge_amd.models.resnet import KvResNet50, init_resnet50

    assert ops.load(), "native kvedge library must be loaded on the GPU box"
    ref = init_resnet50(seed=0)
    return ref, KvResNet50(ref, "cuda")


@pytest.mark.parametrize("B", [1, 8, 64])
def test_edge_graph_vs_fp32_module(models, B):
    from kvedge_amd.models.layers import frames_to_nchw

    ref, kv = models
    eng = InferenceEngine(kv, B, 224, device="cuda", seed=11, use_graph=True,
                          streams=edge_streams(B))
    eng.prepare(warmup=1, autotune=True)
    assert eng.graph is not None and eng.tuning
    torch.cuda.synchronize()
    assert ops._WS, "the edge batches must run split-K layers (workspace allocated)"
    for ws in ops._WS.values():
        ws.fill_(float("nan"))
    eng.run()
    torch.cuda.synchronize()
    probs = eng.outputs[0].float().cpu()
    frames = eng.frames.cpu()  # the frames this replay synthesised
    assert torch.isfinite(probs).all(), "a split-K slab read stale (poisoned) workspace"
    with torch.no_grad():
        lg = kv.raw_outputs(eng.frames).float().cpu()  # same tiles, eager
        lg_ref = ref(frames_to_nchw(frames)).float()
        r16 = copy.deepcopy(ref).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
        x16 = frames_to_nchw(frames).cuda().to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        lg_t16 = r16(x16).float().cpu()
    assert torch.allclose(probs, torch.softmax(lg, 1), rtol=1e-3, atol=1e-6)
    cos = torch.nn.functional.cosine_similarity(lg.flatten(), lg_ref.flatten(), dim=0)
    assert cos > 0.99, (B, float(cos))
    agree = float((lg.argmax(1) == lg_ref.argmax(1)).float().mean())
    agree_t = float((lg_t16.argmax(1) == lg_ref.argmax(1)).float().mean())
    assert agree >= min(0.95, agree_t - 1.0 / B), (B, agree, agree_t)
    # per image (at B = 1 the rate bound above is vacuous): the top-1
    # matches fp32, or PyTorch's own bf16 path flips the same image too, or the fp32 margin
    # is inside the bf16 noise of a logit difference (4 x sqrt(2) x the per-logit rms error)
    top2 = lg_ref.topk(2, dim=1).values
    noise = 4 * float((lg - lg_ref).pow(2).mean().sqrt()) * 2 ** 0.5
    for i in range(B):
        if int(lg[i].argmax()) == int(lg_ref[i].argmax()):
            continue
        margin = float(top2[i, 0] - top2[i, 1])
        assert int(lg_t16[i].argmax()) != int(lg_ref[i].argmax()) or margin < noise, (
            B, i, margin, noise)


@pytest.mark.parametrize("B", [1, 16])
def test_fused_edge_head_matches_unfused(models, B):
    _, kv = models
    fr = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(B)).cuda()
    old = kv.fuse_head
    try:
        with torch.no_grad():
            kv.fuse_head = False
            plain = kv.raw_outputs(fr).float().cpu()
            kv.fuse_head = True
            fused = kv.raw_outputs(fr).float().cpu()
    finally:
        kv.fuse_head = old
    assert fused.shape == plain.shape == (B, 1000)
    cos = torch.nn.functional.cosine_similarity(fused.flatten(), plain.flatten(), dim=0)
    # same bf16 pooled vector; only the fc accumulation order differs
    assert cos > 0.9999, float(cos)
    top2 = plain.topk(2, dim=1).values
    flips = (fused.argmax(1) != plain.argmax(1)).nonzero().flatten().tolist()
    assert all(float(top2[i, 0] - top2[i, 1]) < 0.01 * float(plain.std()) for i in flips), flips
