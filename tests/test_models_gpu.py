"""T-model: deployed models on the HIP kernels vs the CPU reference path and the fp32 nn.Module."""
import pytest
import torch

from kvedge_amd import ops
from kvedge_amd.engine import InferenceEngine
from kvedge_amd.models.layers import frames_to_nchw
from kvedge_amd.models.resnet import KvResNet50, init_resnet50

pytestmark = pytest.mark.gpu


def _close(got, ref):
    """max |err| <= 2% of max |ref| AND relative RMS <= 4e-3."""
    got, ref = got.float(), ref.float()
    err = (got - ref).abs().max().item()
    rr = ((got - ref).pow(2).mean().sqrt() / ref.pow(2).mean().sqrt().clamp_min(1e-12)).item()
    assert err <= 0.02 * ref.abs().max().item() and rr <= 4e-3, (err, rr)


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
        lg_gpu = kv.logits(kv.preprocess(fr.cuda())).float().cpu()
        lg_cpu = kv_cpu.logits(kv_cpu.preprocess(fr)).float()
        lg_ref = ref(frames_to_nchw(fr)).float()
    cos_dep = torch.nn.functional.cosine_similarity(lg_gpu.flatten(), lg_cpu.flatten(), dim=0)
    cos_ref = torch.nn.functional.cosine_similarity(lg_gpu.flatten(), lg_ref.flatten(), dim=0)
    assert cos_dep > 0.995, float(cos_dep)
    assert cos_ref > 0.99, float(cos_ref)


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


@pytest.fixture(scope="module")
def yolo():
    from kvedge_amd.models.yolov8 import KvYoloV8n, init_yolov8n

    ref = init_yolov8n(seed=0)
    return ref, KvYoloV8n(ref, "cuda"), KvYoloV8n(ref, "cpu")


def test_yolov8n_parity(yolo):
    from kvedge_amd.models.yolov8 import frames_to_yolo

    ref, kv, kv_cpu = yolo
    fr = _frames(2, 5, hw=320)
    with torch.no_grad():
        hg = kv.heads(kv.preprocess(fr.cuda()))
        hc = kv_cpu.heads(kv_cpu.preprocess(fr))
        hr = ref(frames_to_yolo(fr))
    for g, c, r in zip(hg, hc, hr):
        g = g.float().cpu()
        cos_dep = torch.nn.functional.cosine_similarity(g.flatten(), c.float().flatten(), dim=0)
        cos_ref = torch.nn.functional.cosine_similarity(
            g.flatten(), r.permute(0, 2, 3, 1).flatten(), dim=0)
        assert cos_dep > 0.999 and cos_ref > 0.995, (float(cos_dep), float(cos_ref))


def test_yolov8n_pipeline_graph(yolo):
    _, kv, _ = yolo
    eng = InferenceEngine(kv, 4, 640, device="cuda", seed=1).prepare(warmup=1)
    dets, cnt = eng.run()
    torch.cuda.synchronize()
    assert dets.shape == (4, 300, 6) and cnt.shape == (4,)
    assert int(cnt.max()) <= 300 and int(cnt.min()) >= 0
    # NMS on the same decoded boxes: GPU kernel == CPU reference
    frames = eng.frames.clone()
    x = kv.preprocess(frames)
    b, s, c = ops.yolo_decode(kv.heads(x), (8, 16, 32), 80)
    o_g, n_g = ops.nms(b, s, c, 0.05, 0.7, 300)
    o_c, n_c = ops.nms(b.cpu(), s.cpu(), c.cpu(), 0.05, 0.7, 300)
    assert torch.equal(n_g.cpu(), n_c)
    assert (o_g.cpu() - o_c).abs().max() < 1e-3


@pytest.mark.parametrize("hw", [(64, 96), (22, 10), (30, 44), (18, 132)])
def test_stem_from_frames_kernel(hw):
    """Frames-in v4 kernel (preprocess + s2d + 2x2 stem in one pass) vs the CPU reference."""
    from kvedge_amd.models.yolov8 import KvYoloV8n, init_yolov8n

    kv = KvYoloV8n(init_yolov8n(seed=1, calibrate=False), "cpu")
    b = kv.b0_frames
    fr = torch.randint(0, 256, (3, hw[0], hw[1], 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(7))
    ref = ops.stem_from_frames(fr, b.spec, b.w, b.b).float()
    got = ops.stem_from_frames(fr.cuda(), b.spec, b.w.cuda(), b.b.cuda())
    torch.cuda.synchronize()
    _close(got.cpu(), ref)


def test_yolov8n_fused_stem_parity(yolo):
    _, kv, kv_cpu = yolo
    fr = _frames(2, 6, hw=320)
    with torch.no_grad():
        hg = kv.heads(kv.stem(fr.cuda()), stem_done=True)
        hc = kv_cpu.heads(kv_cpu.preprocess(fr))
    for g, c in zip(hg, hc):
        cos = torch.nn.functional.cosine_similarity(g.float().cpu().flatten(), c.float().flatten(),
                                                    dim=0)
        assert cos > 0.999, float(cos)


@pytest.mark.parametrize("hw,n", [((224, 224), 5), ((64, 96), 5), ((36, 20), 5), ((224, 224), 40),
                                  ((36, 20), 160)])
def test_stem_pool_frames_kernel(resnet, hw, n):
    """Frames-in ResNet stem + pool (preprocess fused into the fetch) vs the CPU reference
    preprocess -> s2d stem -> pool; borders (padding must be 0, not -mean/std) included.
    n = 40 / 160: more bands than CUs, so workgroups walk band ranges (shared stem row)."""
    _, kv, kv_cpu = resnet
    fr = torch.randint(0, 256, (n, hw[0], hw[1], 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(11))
    s = kv_cpu.stem
    ref = ops.stem_pool_frames(fr, s.spec, s.w, s.b).float()
    got = ops.stem_pool_frames(fr.cuda(), kv.stem.spec, kv.stem.w, kv.stem.b)
    two = ops.stem_pool(ops.preprocess(fr.cuda(), s2d=True), kv.stem.spec, kv.stem.w, kv.stem.b)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    _close(got.cpu(), ref)
    err2 = (got.float() - two.float()).abs().max().item()
    assert err2 <= 0.01 * ref.abs().max().item() + 0.01, err2


def test_resnet50_frames_in_parity(resnet):
    """The default GPU forward (frames straight into the stem kernel) equals the
    explicit preprocess path."""
    _, kv, _ = resnet
    fr = _frames(4, 3).cuda()
    with torch.no_grad():
        lg_fused = kv.raw_outputs(fr).float()
        lg_two = kv.logits(kv.preprocess(fr)).float()
    torch.cuda.synchronize()
    # logits, not 1000-way probabilities (~1e-3 each, where an atol says nothing).  The two
    # paths use different stems (12-channel s2d K 192 vs 16-channel K 256), so they differ
    # by bf16 rounding carried through 50 layers (cos > 0.9995 is relative RMS < ~3 %)
    cos = torch.nn.functional.cosine_similarity(lg_fused.flatten(), lg_two.flatten(), dim=0)
    assert cos > 0.9995, float(cos)
    d = lg_fused - lg_two
    assert d.abs().max() <= 3e-2 * lg_two.abs().max(), d.abs().max()
    assert torch.equal(lg_fused.argmax(1), lg_two.argmax(1))


@pytest.mark.parametrize("mb,nb", [(2, 3), (4, 2), (2, 5)])
def test_resnet50_microbatch_fused_tail(resnet, mb, nb):
    """Micro-batched early stages (fused tails inside the micro-batch, the last one
    writing y and the next conv1 output into full-batch slices) == the whole-batch path."""
    _, kv, _ = resnet
    fr = _frames(8, 5).cuda()
    with torch.no_grad():
        lg_full = kv.logits(fr, frames_in=True).float()
        kv.microbatch, kv.microbatch_blocks = mb, nb
        try:
            lg_mb = kv.logits(fr, frames_in=True).float()
        finally:
            kv.microbatch, kv.microbatch_blocks = 0, 3
    torch.cuda.synchronize()
    assert torch.allclose(lg_full, lg_mb, atol=1e-2, rtol=1e-2), (lg_full - lg_mb).abs().max()


def test_resnet50_microbatch_seam_gate_uses_full_batch(resnet, monkeypatch):
    """the seam gate of the micro-batched blocks is evaluated on the FULL
    batch.  With SEAM_MIN_WGS between the micro-batch's and the full batch's workgroup
    counts (8 images at 28x28: 49 workgroups of 128 rows; micro-batch 2: 13), both paths
    must fuse the same stage-2 boundary and give the same logits."""
    _, kv, _ = resnet
    monkeypatch.setattr(ops, "SEAM_MIN_WGS", 20)
    fr = _frames(8, 6).cuda()
    with torch.no_grad():
        lg_full = kv.logits(fr, frames_in=True).float()
        kv.microbatch, kv.microbatch_blocks = 2, 5
        try:
            lg_mb = kv.logits(fr, frames_in=True).float()
        finally:
            kv.microbatch, kv.microbatch_blocks = 0, 3
    torch.cuda.synchronize()
    assert torch.allclose(lg_full, lg_mb, atol=1e-2, rtol=1e-2), (lg_full - lg_mb).abs().max()


@pytest.mark.parametrize("hw,n", [((224, 224), 3), ((64, 96), 5), ((38, 20), 5), ((224, 224), 40),
                                  ((36, 20), 300), ((22, 28), 7)])
def test_stem12_pool_frames_kernel(resnet, hw, n):
    """12-channel s2d stem (csrc/kernels/stem12.hip, K 192) vs its CPU reference step for
    step, and vs the fp32 nn.Conv2d stem: odd stem heights (38 -> 19 rows), image-start
    bands inside a workgroup's range (n = 300: more bands than workgroups), a channel-slice
    output with a NaN canary outside it."""
    ref, kv, kv_cpu = resnet
    fr = torch.randint(0, 256, (n, hw[0], hw[1], 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(13))
    want = ops.stem12_reference(fr, kv_cpu.stem12_w, kv_cpu.stem.b)
    Hp, Wp = want.shape[1], want.shape[2]
    out = torch.full((n, Hp, Wp, 80), float("nan"), dtype=torch.bfloat16, device="cuda")
    ops.stem12_pool_frames(fr.cuda(), kv.stem12_w, kv.stem.b, out=out, y_coff=8)
    torch.cuda.synchronize()
    got = out.cpu()
    assert torch.isnan(got[..., :8].float()).all() and torch.isnan(got[..., 72:].float()).all()
    _close(got[..., 8:72], want)
    # and the model's own stem (fp32 nn.Module conv + BN + ReLU + pool)
    with torch.no_grad():
        x = frames_to_nchw(fr)
        r = torch.nn.functional.max_pool2d(torch.relu(ref.bn1(ref.conv1(x))), 3, 2, 1)
    r = r.permute(0, 2, 3, 1)
    cos = torch.nn.functional.cosine_similarity(got[..., 8:72].float().flatten(), r.flatten(), dim=0)
    assert cos > 0.999, float(cos)


@pytest.mark.parametrize("n,hw", [(3, (64, 96)), (2, (640, 640)), (1, (4, 32)), (7, (128, 640)),
                                  (40, (128, 96)), (5, (36, 64))])
def test_yolo_stem2_kernel(n, hw):
    """Fused YOLO b0 + b1 from raw frames (csrc/kernels/yolo_stem2.hip) vs the two reference
    ops in sequence: band ranges that start mid-image (n = 7: one band per workgroup,
    H1 = 32) and cross image boundaries (n = 40), the full 640^2 shape, a single band."""
    from kvedge_amd.models.yolov8 import KvYoloV8n, init_yolov8n

    kv = KvYoloV8n(init_yolov8n(seed=2, calibrate=False), "cpu")
    b0, b1 = kv.b0_frames, kv.b1
    fr = torch.randint(0, 256, (n, hw[0], hw[1], 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(17))
    ref = ops.yolo_stem2(fr, b0.spec, b0.w, b0.b, b1.spec, b1.w, b1.b).float()
    got = ops.yolo_stem2(fr.cuda(), b0.spec, b0.w.cuda(), b0.b.cuda(), b1.spec, b1.w.cuda(),
                         b1.b.cuda())
    torch.cuda.synchronize()
    assert got.shape == ref.shape == (n, hw[0] // 4, hw[1] // 4, 32)
    _close(got.cpu(), ref)


def test_yolov8n_fused_stem_b1_parity(yolo):
    """Fused b0 + b1 (yolo_stem2) through the whole network vs the CPU model, judged against
    the unfused GPU path (frames-in b0 kernel, then the b1 conv tile) on the SAME frames:
    random-init heads carry bf16 rounding through ~60 layers, so the absolute cosine depends
    on the frames (0.9988 on this seed); the fused path must be as close as the unfused one."""
    _, kv, kv_cpu = yolo
    fr = _frames(2, 8, hw=320)
    cs = torch.nn.functional.cosine_similarity
    with torch.no_grad():
        hg = kv.heads(kv.stem_b1(fr.cuda()), b1_done=True)
        hu = kv.heads(kv.stem(fr.cuda()), stem_done=True)
        hc = kv_cpu.heads(kv_cpu.preprocess(fr))
    for g, u, c in zip(hg, hu, hc):
        g, u, c = g.float().cpu().flatten(), u.float().cpu().flatten(), c.float().flatten()
        cg, cu = float(cs(g, c, dim=0)), float(cs(u, c, dim=0))
        assert cg > 0.998 and cg >= cu - 5e-4, (cg, cu)
        assert float(cs(g, u, dim=0)) > 0.999


