"""Fused 64-wide bottleneck body (csrc/kernels/conv_block.hip) vs the plain-PyTorch fp32
reference of the same three convs (kvedge_amd.ops.conv_block on CPU tensors): residual and
fused-downsample forms, both tail widths, row/image tails (W < 64, odd H/W for the 3x3
padding, workgroup row ranges crossing images), and a NaN-poisoned output canary."""
import pytest
import torch

from kvedge_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert ops.load(), "native kvedge library must be loaded on the GPU box"


def _inputs(N, H, W, nt, dual, seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(N, H, W, 64, generator=g).relu().to(torch.bfloat16)
    w2 = (torch.randn(64, 576, generator=g) * (2.0 / 576) ** 0.5).to(torch.bfloat16)
    b2 = torch.randn(64, generator=g) * 0.1
    k3 = 128 if dual else 64
    w3 = (torch.randn(256, k3, generator=g) * (2.0 / k3) ** 0.5).to(torch.bfloat16)
    b3 = torch.randn(256, generator=g) * 0.1
    w1 = (torch.randn(nt, 256, generator=g) * (2.0 / 256) ** 0.5).to(torch.bfloat16)
    b1 = torch.randn(nt, generator=g) * 0.1
    extra = torch.randn(N, H, W, 64 if dual else 256, generator=g).to(torch.bfloat16)
    return t, w2, b2, w3, b3, w1, b1, extra


def _close(got, ref, what):
    got, ref = got.float(), ref.float()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    rr = ((got - ref).pow(2).mean().sqrt() / ref.pow(2).mean().sqrt().clamp_min(1e-12)).item()
    assert err <= 0.02 * scale and rr <= 4e-3, (what, err, scale, rr)


@pytest.mark.parametrize("dual", [False, True])
@pytest.mark.parametrize("nt", [64, 128])
@pytest.mark.parametrize("shape", [(2, 56, 56), (3, 13, 11), (1, 1, 1), (5, 7, 9), (3, 2, 64),
                                   (300, 3, 5)])
def test_conv_block_vs_reference(dual, nt, shape):
    """Shapes: the ResNet stage-1 row (W = 56), odd H/W (padding columns), a single pixel,
    H = 2 (every row is an image's first or last), W = 64 (a full tile row), and more
    images than CUs (workgroup row ranges that start and end mid-image)."""
    N, H, W = shape
    t, w2, b2, w3, b3, w1, b1, extra = _inputs(N, H, W, nt, dual, seed=N * 100 + H + nt)
    kw = {"x2": extra} if dual else {"res": extra}
    y_ref, z_ref = ops.conv_block(t, w2, b2, w3, b3, w1, b1, **kw)
    dev = [a.cuda() for a in (t, w2, b2, w3, b3, w1, b1)]
    kwd = {k: v.cuda() for k, v in kw.items()}
    if dual and nt == 128:  # 128-wide tail weights + both resident conv3 blocks > 160 KiB LDS
        with pytest.raises(RuntimeError):
            ops.conv_block(*dev, **kwd)
        return
    y, z = ops.conv_block(*dev, **kwd)
    torch.cuda.synchronize()
    _close(y.cpu(), y_ref, "y")
    _close(z.cpu(), z_ref, "z")


def test_conv_block_poisoned_canary():
    """Outputs written into NaN-filled buffers with NaN tails: every output element finite,
    nothing written past the tensors (M = 3*13*11 = 429 is not a multiple of the tile)."""
    N, H, W, nt = 3, 13, 11, 64
    t, w2, b2, w3, b3, w1, b1, res = [a.cuda() for a in _inputs(N, H, W, nt, False, seed=7)]
    m = N * H * W
    fy = torch.full((m * 256 + 4096,), float("nan"), dtype=torch.bfloat16, device="cuda")
    fz = torch.full((m * nt + 4096,), float("nan"), dtype=torch.bfloat16, device="cuda")
    y = fy[:m * 256].view(N, H, W, 256)
    z = fz[:m * nt].view(N, H, W, nt)
    ops.conv_block(t, w2, b2, w3, b3, w1, b1, res=res, out=y, z=z)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all() and torch.isfinite(z).all()
    assert torch.isnan(fy[m * 256:].float()).all() and torch.isnan(fz[m * nt:].float()).all()


def test_conv_block_rejects_bad_forms():
    t, w2, b2, w3, b3, w1, b1, res = [a.cuda() for a in _inputs(1, 4, 4, 64, False, seed=1)]
    with pytest.raises(RuntimeError):  # neither residual nor downsample source
        ops.conv_block(t, w2, b2, w3, b3, w1, b1)
    with pytest.raises(RuntimeError):  # tail width other than 64 / 128
        ops.conv_block(t, w2, b2, w3, b3, w1[:32].contiguous(), b1[:32].contiguous(), res=res)
    t2, w2, b2, w3, b3, w1, b1, res2 = [a.cuda() for a in _inputs(1, 2, 65, 64, False, seed=2)]
    with pytest.raises(RuntimeError):  # rows wider than one 64-pixel tile
        ops.conv_block(t2, w2, b2, w3, b3, w1, b1, res=res2)
