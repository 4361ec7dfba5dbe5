"""CPU tests of the op layer: weight packing, conv specs, reference semantics."""
import pytest
import torch
import torch.nn.functional as F

from kvedge_amd import ops
from kvedge_amd.ops import ConvSpec


@pytest.mark.parametrize("cin,cout,k,stride,pad", [
    (64, 128, 3, 1, 1), (3, 64, 7, 2, 3), (3, 16, 3, 2, 1), (256, 512, 1, 2, 0),
    (48, 32, 1, 1, 0), (16, 16, 3, 1, 1)])
def test_pack_unpack_roundtrip(cin, cout, k, stride, pad):
    spec = ConvSpec.auto(cin, cout, k, stride, pad)
    w = torch.randn(cout, cin, k, k)
    wp = ops.pack_conv_weight(w, spec)
    assert wp.shape == (cout, spec.Kpad) and wp.dtype == torch.bfloat16
    assert spec.Kpad % 64 == 0 and spec.Kpad >= spec.K
    wu = ops.unpack_conv_weight(wp, spec)
    assert torch.equal(wu, w.to(torch.bfloat16).float())
    # padding region is zero
    assert wp[:, spec.K:].abs().sum() == 0


def test_spec_modes():
    assert ConvSpec.auto(3, 64, 7, 2, 3).mode == ops.MODE_STEM
    assert ConvSpec.auto(64, 64, 1, 1, 0).mode == ops.MODE_GEMM
    assert ConvSpec.auto(64, 64, 1, 2, 0).mode == ops.MODE_GENERAL
    assert ConvSpec.auto(64, 64, 3).mode == ops.MODE_GENERAL
    s = ConvSpec.auto(3, 64, 7, 2, 3)
    assert s.K == 7 * 8 * 4 and s.Kpad == 256 and s.cin_eff == 4
    assert s.out_hw(224, 224) == (112, 112)


def test_reference_conv_matches_torch_and_slices():
    spec = ConvSpec.auto(32, 48, 3, 2, 1, ops.ACT_RELU)
    x = torch.randn(2, 9, 9, 64).to(torch.bfloat16)
    w = torch.randn(48, 32, 3, 3) * 0.1
    b = torch.randn(48)
    wp = ops.pack_conv_weight(w, spec)
    out = torch.zeros(2, 5, 5, 80, dtype=torch.bfloat16)
    ops.conv2d(x, spec, wp, b, out=out, x_coff=16, y_coff=16)
    ref = F.conv2d(x[..., 16:48].float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(), b,
                   2, 1).relu().permute(0, 2, 3, 1)
    assert (out[..., 16:64].float() - ref).abs().max() < 0.05
    assert out[..., :16].abs().sum() == 0 and out[..., 64:].abs().sum() == 0


def test_stem_reference_ignores_pad_channel():
    spec = ConvSpec.auto(3, 8, 7, 2, 3)
    g = torch.Generator().manual_seed(0)
    x4 = torch.randn(1, 16, 16, 4, generator=g).to(torch.bfloat16)
    x4[..., 3] = 0
    w = torch.randn(8, 3, 7, 7, generator=g) * 0.1
    y = ops.conv2d(x4, spec, ops.pack_conv_weight(w, spec), None)
    ref = F.conv2d(x4[..., :3].float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(),
                   None, 2, 3).permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max() < 0.01 * ref.abs().max() + 1e-3


def test_synth_frames_deterministic():
    a = torch.empty(2, 8, 8, 3, dtype=torch.uint8)
    b = torch.empty_like(a)
    ops.synth_frames(a, 1, 5)
    ops.synth_frames(b, 1, 5)
    assert torch.equal(a, b)
    ops.synth_frames(b, 1, 6)
    assert not torch.equal(a, b)
    ctr = torch.tensor([5])
    ops.synth_frames(b, 1, ctr)
    assert torch.equal(a, b) and int(ctr) == 6
    ctr2 = torch.tensor([5, 0])  # [counter, done-count] (the engine's in-kernel bump form)
    ops.synth_frames(b, 1, ctr2)
    assert torch.equal(a, b) and ctr2.tolist() == [6, 0]
    # bytes look uniform
    big = torch.empty(4, 64, 64, 3, dtype=torch.uint8)
    ops.synth_frames(big, 0, 0)
    assert abs(big.float().mean().item() - 127.5) < 3


def test_pools_softmax_reference():
    x = torch.randn(2, 8, 8, 16).to(torch.bfloat16)
    y = ops.maxpool2d(x, 3, 2, 1)
    assert y.shape == (2, 4, 4, 16)
    buf = torch.zeros(1, 6, 6, 32, dtype=torch.bfloat16)
    buf[..., :8] = torch.randn(1, 6, 6, 8).to(torch.bfloat16)
    ops.sppf_pool(buf, 8)
    # mp13 over a 6x6 map = global max per channel
    assert torch.equal(buf[..., 24:32].amax((1, 2)), buf[..., :8].amax((1, 2)))
    p, am = ops.softmax_rows(torch.randn(3, 10).to(torch.bfloat16))
    assert torch.allclose(p.sum(1), torch.ones(3)) and am.shape == (3,)


def test_reference_nms_simple():
    boxes = torch.tensor([[[0, 0, 10, 10], [1, 1, 11, 11], [50, 50, 60, 60], [0, 0, 10, 10]]],
                         dtype=torch.float32)
    scores = torch.tensor([[0.9, 0.8, 0.7, 0.95]])
    cls = torch.tensor([[0, 0, 0, 1]], dtype=torch.int32)
    out, cnt = ops.nms(boxes, scores, cls, conf=0.25, iou=0.5, max_det=10)
    # box 3 (cls 1) kept first, box 0 kept, box 1 suppressed by 0, box 2 kept
    assert int(cnt[0]) == 3
    assert out[0, 0, 4].item() == pytest.approx(0.95)
    assert out[0, 1, 4].item() == pytest.approx(0.9)
    assert out[0, 2, 4].item() == pytest.approx(0.7)


def test_gpu_path_fails_loudly_without_library(monkeypatch):
    monkeypatch.setattr(ops, "_loaded", False)
    monkeypatch.setattr(ops, "_LIB_PATH", "/nonexistent/_C.so")
    with pytest.raises(RuntimeError, match="native kernels are required"):
        ops._native()


def test_s2d_stem_equals_strided_conv():
    """Stride-2 stem == stride-1 conv over the space-to-depth input (ResNet 7x7/3 and YOLO 3x3/1)."""
    import torch.nn as nn
    from kvedge_amd.models.layers import DeployedConv

    for k, p, cout, hw in ((7, 3, 8, 32), (3, 1, 16, 32)):
        conv = nn.Conv2d(3, cout, k, 2, p, bias=False)
        fr = torch.randint(0, 256, (2, hw, hw, 3), dtype=torch.uint8)
        d = DeployedConv.stem_s2d(conv, None, ops.ACT_NONE)
        xs = ops.preprocess(fr, s2d=True)
        assert xs.shape == (2, hw // 2, hw // 2, 16)
        y = d(xs).float()
        x4 = ops.preprocess(fr).float()[..., :3].permute(0, 3, 1, 2)
        ref = F.conv2d(x4, conv.weight.detach().to(torch.bfloat16).float(), None, 2, p)
        assert y.shape == ref.permute(0, 2, 3, 1).shape
        assert (y - ref.permute(0, 2, 3, 1)).abs().max() < 0.05 * ref.abs().max() + 0.05


def test_c2f16_reference_matches_block():
    """ops.c2f16's CPU reference is the DC2f four-conv path (same bf16 intermediates)."""
    import torch
    from kvedge_amd import ops
    from kvedge_amd.models.yolov8 import C2f, DC2f
    torch.manual_seed(1)
    blk = DC2f(C2f(32, 32, 1, True).eval(), "cpu")
    x = (torch.randn(1, 8, 16, 40) * 2).to(torch.bfloat16)
    four = blk(x, x_coff=8)
    b1, b2, _ = blk.m[0]
    one = ops.c2f16(x, blk.cv1.w, blk.cv1.b, b1.w, b1.b, b2.w, b2.b, blk.cv2.w, blk.cv2.b,
                    x_coff=8)
    assert torch.equal(four, one)


def test_conv_dual2_up2_reference_matches_upsample_concat():
    """ops.conv_dual2 with up2 (the neck's upsample + concat folded into cv1) equals the
    1x1 conv over the materialised [upsample2x(low) | skip] concat, weights permuted."""
    import torch
    from kvedge_amd import ops
    from kvedge_amd.ops import ConvSpec
    g = torch.Generator().manual_seed(4)
    N, H, W, c_up, c_skip, cout = 2, 6, 8, 128, 64, 72
    low = (torch.randn(N, H // 2, W // 2, 8 + c_up, generator=g)).to(torch.bfloat16)
    skip = (torch.randn(N, H, W, 16 + c_skip, generator=g)).to(torch.bfloat16)
    spec = ConvSpec.auto(c_up + c_skip, cout, 1, 1, 0, ops.ACT_SILU)
    w = ops.pack_conv_weight(torch.randn(cout, c_up + c_skip, 1, 1, generator=g) * 0.05, spec)
    b = torch.randn(cout, generator=g)
    cat = torch.cat([low[..., 8:].repeat_interleave(2, 1).repeat_interleave(2, 2),
                     skip[..., 16:]], -1)
    ref = ops.conv2d(cat, spec, w, b)
    wd = torch.cat([w[:, c_up:], w[:, :c_up]], 1).contiguous()
    out = torch.zeros(N, H, W, cout + 8, dtype=torch.bfloat16)
    ops.conv_dual2(skip, c_skip, low, wd, b, ops.ACT_SILU, out, x_coff=16, x2_coff=8, y_coff=8,
                   up2=True)
    assert (out[..., :8] == 0).all()
    assert (out[..., 8:].float() - ref.float()).abs().max() <= 0.02 * ref.float().abs().max()


def test_c2f_up_call_matches_upsample_path():
    """DC2f.up_call (cv1 as the up2 dual GEMM) == upsample2x into the concat + the block."""
    import torch
    from kvedge_amd import ops
    from kvedge_amd.models.yolov8 import C2f, DC2f
    torch.manual_seed(2)
    blk = DC2f(C2f(192, 64, 1, False).eval(), "cpu")
    N, H, W = 1, 8, 6
    low = torch.randn(N, H // 2, W // 2, 192).to(torch.bfloat16)      # up source at channel 64
    cat = torch.randn(N, H, W, 192).to(torch.bfloat16)               # [up 128 | skip 64]
    ops.upsample2x(low, cat, C=128, x_coff=64, y_coff=0)
    ref = blk(cat)
    got = blk.up_call(cat, 128, low, 64, 128)
    d = (got.float() - ref.float()).abs().max().item()
    assert d <= 0.03 * ref.float().abs().max().item(), d
