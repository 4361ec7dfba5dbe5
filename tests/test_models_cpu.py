"""CPU tests: BN folding, deployed ResNet-50 vs the fp32 module, engine plumbing."""
import pytest
import torch
import torch.nn as nn

from kvedge_amd import ops
from kvedge_amd.engine import InferenceEngine
from kvedge_amd.models.layers import DeployedConv, fold_bn, frames_to_nchw
from kvedge_amd.models.resnet import KvResNet50, init_resnet50


def test_fold_bn_exact():
    torch.manual_seed(0)
    conv = nn.Conv2d(8, 16, 3, 1, 1, bias=False)
    bn = nn.BatchNorm2d(16)
    bn.running_mean.uniform_(-1, 1)
    bn.running_var.uniform_(0.5, 2)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-1, 1)
    bn.eval()
    x = torch.randn(2, 8, 10, 10)
    w, b = fold_bn(conv, bn)
    y = nn.functional.conv2d(x, w, b, 1, 1)
    assert torch.allclose(y, bn(conv(x)), atol=1e-5)


def test_deployed_conv_from_modules():
    conv = nn.Conv2d(16, 32, 3, 2, 1, bias=False)
    bn = nn.BatchNorm2d(16 * 2).eval()
    d = DeployedConv.from_modules(conv, bn, ops.ACT_RELU)
    assert d.spec.stride == 2 and d.spec.pad == 1 and d.w.shape == (32, d.spec.Kpad)
    assert d.flops_per_pixel == 2 * 9 * 16 * 32


def test_resnet50_cpu_deployed_vs_module():
    ref = init_resnet50(seed=0)
    kv = KvResNet50(ref, "cpu")
    # stem + bottleneck convs + downsamples + fused conv3/downsample GEMMs + fc
    assert len(kv.convs()) == 1 + 16 * 3 + 4 + 4 + 1
    assert abs(kv.flops_per_image() / 1e9 - 8.18) < 0.05
    fr = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        lg = kv.logits(kv.preprocess(fr)).float()
        lr = ref(frames_to_nchw(fr))
    cos = nn.functional.cosine_similarity(lg.flatten(), lr.flatten(), dim=0)
    assert cos > 0.98, float(cos)


def test_engine_cpu_eager():
    class Tiny:
        def __call__(self, frames):
            x = ops.preprocess(frames)
            pooled = x.float().mean((1, 2))
            return ops.softmax_rows(pooled.to(torch.bfloat16))

    eng = InferenceEngine(Tiny(), 2, 16, device="cpu", seed=1).prepare(warmup=1)
    assert eng.graph is None
    p1 = eng.run()[0].clone()
    p2 = eng.run()[0].clone()
    assert p1.shape == (2, 4) and not torch.equal(p1, p2)
    assert eng.run_timed(2) >= 0
    st = eng.measure_latency(3)
    assert st.count == 3 and st.percentile(50) >= 0


def test_yolov8n_cpu_structure_and_parity():
    from kvedge_amd.models.yolov8 import KvYoloV8n, frames_to_yolo, init_yolov8n

    ref = init_yolov8n(seed=0)
    assert abs(sum(p.numel() for p in ref.parameters()) - 3_157_184) == 0
    kv = KvYoloV8n(ref, "cpu")
    assert abs(kv.flops_per_image() / 1e9 - 8.74) < 0.02
    fr = torch.randint(0, 256, (1, 256, 256, 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        hk = kv.heads(kv.preprocess(fr))
        hr = ref(frames_to_yolo(fr))
    for k, r in zip(hk, hr):
        assert k.shape == r.permute(0, 2, 3, 1).shape
        cos = nn.functional.cosine_similarity(k.float().flatten(), r.permute(0, 2, 3, 1).flatten(),
                                              dim=0)
        assert cos > 0.995, float(cos)
    dets, cnt = kv(fr)
    assert dets.shape == (1, 300, 6) and 0 <= int(cnt[0]) <= 300


def test_residual_after_activation_flag():
    from kvedge_amd.ops import ConvSpec

    spec = ConvSpec.auto(16, 16, 3, 1, 1, ops.ACT_SILU | ops.RES_AFTER_ACT)
    x = torch.randn(1, 5, 5, 16).to(torch.bfloat16)
    w = torch.randn(16, 16, 3, 3) * 0.1
    r = torch.randn(1, 5, 5, 16).to(torch.bfloat16)
    y = ops.conv2d(x, spec, ops.pack_conv_weight(w, spec), torch.zeros(16), res=r)
    conv = nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(),
                                None, 1, 1).permute(0, 2, 3, 1)
    ref = nn.functional.silu(conv) + r.float()
    assert (y.float() - ref).abs().max() < 0.05


def test_resnet50_microbatch_equivalence():
    ref = init_resnet50(seed=1, calibrate=False)
    kv = KvResNet50(ref, "cpu")
    fr = torch.randint(0, 256, (4, 64, 64, 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        x = kv.preprocess(fr)
        full = kv.features(x).float()
        kv.microbatch, kv.microbatch_blocks = 2, 4
        micro = kv.features(x).float()
    assert torch.equal(full, micro)


def test_yolo_frames_in_stem_matches_preprocess_path():
    """ops.stem_from_frames (1/255 folded into the weights, raw 0..255 inputs) == the
    unfused preprocess -> s2d stem conv, on the CPU reference ops."""
    from kvedge_amd.models.yolov8 import KvYoloV8n, init_yolov8n

    kv = KvYoloV8n(init_yolov8n(seed=1, calibrate=False), "cpu")
    fr = torch.randint(0, 256, (2, 64, 96, 3), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(4))
    with torch.no_grad():
        fused = kv.stem(fr).float()
        plain = kv.b0(kv.preprocess(fr)).float()
    assert fused.shape == plain.shape == (2, 32, 48, 16)
    assert (fused - plain).abs().max().item() <= 0.02 * plain.abs().max().item() + 0.02


def test_resnet_tail_and_seam_plumbing():
    """Which bottleneck boundaries run fused on the GPU: the stage-1 v3 tails (blocks 0-2)
    and the v9 seams (conv_seam.hip: plain conv3 + residual -> next conv1, stages 2-3 and
    both stage boundaries).  The dual (downsample) blocks 3, 7, 13 and stage 4 stay
    unfused.  On CPU every fused call equals the unfused two-conv composition bit for bit."""
    import torch

    from kvedge_amd import ops
    from kvedge_amd.models.resnet import KvResNet50, init_resnet50

    kv = KvResNet50(init_resnet50(0, calibrate=False), "cpu")
    fused = [i for i, b in enumerate(kv.blocks[:-1]) if b.can_tail(kv.blocks[i + 1])]
    if ops.SEAM_ENABLED:
        assert fused == [0, 1, 2, 4, 5, 6, 8, 9, 10, 11]
    else:
        assert fused == [0, 1, 2]
    g = torch.Generator().manual_seed(1)
    for i in (4, 6, 9):  # seam shapes: stage 2, 2 -> 3, stage 3
        b, nxt = kv.blocks[i], kv.blocks[i + 1]
        k3, cout = b.c3.spec.cin, b.c3.spec.cout
        x = torch.randn(1, 3, 5, cout, generator=g).relu().to(torch.bfloat16)
        t1 = torch.randn(1, 3, 5, k3, generator=g).relu().to(torch.bfloat16)
        c2 = b.c2(t1)
        y_f, z_f = b.call_tail(x, nxt, t1=t1)
        y_u = b.c3(c2, res=x)
        z_u = nxt.c1(y_u)
        assert torch.equal(y_f, y_u) and torch.equal(z_f, z_u), i

def test_engine_streams_cpu_and_split_check():
    from kvedge_amd.engine import _cat_outputs

    class Tiny:
        def __call__(self, frames):
            return ops.softmax_rows(ops.preprocess(frames).float().mean((1, 2)).to(torch.bfloat16))

    # CPU: slicing onto HIP streams collapses to one stream
    eng = InferenceEngine(Tiny(), 4, 16, device="cpu", seed=1, streams=2).prepare(warmup=1)
    assert eng.n_streams == 1 and eng.run()[0].shape == (4, 4)
    with pytest.raises(ValueError):
        InferenceEngine(Tiny(), 3, 16, device="cpu", streams=2)
    a, b = torch.arange(6).view(2, 3), torch.arange(6, 12).view(2, 3)
    assert torch.equal(_cat_outputs([a, b]), torch.arange(12).view(4, 3))
    t = _cat_outputs([(a, a[:, 0]), (b, b[:, 0])])
    assert torch.equal(t[0], torch.arange(12).view(4, 3)) and t[1].tolist() == [0, 3, 6, 9]


def test_op_roofline_flops_match_model():
    """tools/op_roofline.py's per-op FLOPs (derived from each op call's own arguments) sum to
    the reference architecture's FLOPs exactly, so its floors price the real model."""
    import importlib.util
    import os

    from kvedge_amd import ops
    from kvedge_amd.models.yolov8 import KvYoloV8n, init_yolov8n

    path = os.path.join(os.path.dirname(__file__), "..", "tools", "op_roofline.py")
    spec = importlib.util.spec_from_file_location("op_roofline", path)
    R = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(R)
    m = KvYoloV8n(init_yolov8n(seed=0, calibrate=False), "cpu")
    fr = torch.randint(0, 256, (1, 96, 96, 3), dtype=torch.uint8)
    with torch.no_grad():
        rows = R.costs_only(m, fr, ops)
    assert sum(r[2] for r in rows) == m.flops_per_image(96)
    assert rows[0][0].startswith("stem") and rows[-1][0] == "nms"
    assert all(r[1] > 0 for r in rows)
    assert ops.conv2d.__name__ == "conv2d"  # wrappers removed


def test_yolo_detect_pairs_fit_and_match_unfused():
    """Every Detect level's two branches have a fused pair form (ops.conv_pair: 3x3 + SiLU ->
    1x1 kept on chip on the GPU), and the pair's reference equals the two convs it replaces
    (bf16 intermediate) at the level's own slices of the head map."""
    from kvedge_amd.models.yolov8 import KvYoloV8n, init_yolov8n

    kv = KvYoloV8n(init_yolov8n(seed=3, calibrate=False), "cpu")
    for lv, hw in zip(kv.levels, (16, 8, 4)):
        assert all(p.fits for p in lv.pairs)
        cin = lv.stem.spec.cin
        x = (torch.randn(2, hw, hw, cin, generator=torch.Generator().manual_seed(hw))).to(torch.bfloat16)
        s = lv.stem(x)
        z = torch.zeros(2, hw, hw, 144, dtype=torch.bfloat16)
        for pair, xo, zo in ((lv.pairs[0], 0, 0), (lv.pairs[1], lv.ca, 64)):
            pair(s, z, x_coff=xo, z_coff=zo)
        assert torch.equal(z, lv(x))  # the CPU forward runs the unfused convs
