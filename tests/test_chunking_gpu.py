"""Batches past the 2 GiB-per-operand limit of one launch.

The conv kernels address operands through 32-bit buffer offsets, so kv_conv2d splits a
batch whose operands exceed 2 GiB into image-chunk launches.  Tested two ways:
  * the chunk size is shrunk to a few images so EVERY conv family of both models
    (direct / streaming / LDS-DMA / dual downsample / fused tail / frames-in stem) runs
    chunked, and the outputs must equal the single-launch outputs bit for bit;
  * real sizes: ResNet-50 at batch 2048 and YOLOv8n at batch 768 (operands > 2 GiB), with
    the first images' outputs checked against a small-batch run of the same frames.
"""
import pytest
import torch

from kvedge_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert ops.load(), "native kvedge library must be loaded on the GPU box"
    yield
    torch.ops.kvedge.set_conv_chunk_bytes(0)


def _frames(n, hw, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (n, hw, hw, 3), dtype=torch.uint8, generator=g).cuda()


@pytest.mark.parametrize("model", ["resnet50", "yolov8n"])
def test_chunked_launches_bitwise_equal(model):
    if model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50 as M
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n as M
    m = M.build(seed=0, device="cuda", calibrate=False)
    fr = _frames(5, M.image_size)
    with torch.no_grad():
        full = m.raw_outputs(fr).float().clone()
        # one 640x640 YOLO image's largest operand is ~3.3 MB, a ResNet one ~1.6 MB:
        # 4 MB chunks split every conv into 1-3 image launches (5 = 2+2+1 or 1+...)
        assert torch.ops.kvedge.set_conv_chunk_bytes(4 << 20) == 4 << 20
        chunked = m.raw_outputs(fr).float().clone()
        torch.ops.kvedge.set_conv_chunk_bytes(0)
    torch.cuda.synchronize()
    assert torch.isfinite(full).all()
    assert torch.equal(full, chunked)


@pytest.mark.parametrize("model,batch", [("resnet50", 2048), ("yolov8n", 768)])
def test_batch_beyond_2gib_slice_parity(model, batch):
    if model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50 as M
        big_op = batch * 56 * 56 * 256 * 2        # layer1 output
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n as M
        big_op = batch * 320 * 320 * 16 * 2       # stem output
    assert big_op > 2 ** 31  # the single-launch path could not address this
    m = M.build(seed=0, device="cuda", calibrate=False)
    fr = _frames(batch, M.image_size, seed=1)
    with torch.no_grad():
        big = m.raw_outputs(fr)[:8].float().cpu()
        torch.cuda.synchronize()
        small = m.raw_outputs(fr[:8].contiguous()).float().cpu()
    assert torch.isfinite(big).all()
    # same kernels per image; only the chunking differs -> identical up to tile choice
    cos = torch.nn.functional.cosine_similarity(big.flatten(), small.flatten(), dim=0)
    assert cos > 0.9999, float(cos)
    assert (big - small).abs().max() <= 2e-2 * small.abs().max() + 1e-3


def test_conv_dual2_up2_chunked_bitwise_equal():
    """conv_dual2 (the YOLO neck's upsample + concat folded into cv1) has no
    whole-tensor 2 GiB cap any more; past the chunk size it runs as image-chunk launches
    with x2 advanced per (half-size) image, bit-identical to one launch."""
    g = torch.Generator().manual_seed(7)
    N, H, W = 6, 40, 40
    skip = torch.randn(N, H, W, 192, generator=g).to(torch.bfloat16).cuda()
    low = torch.randn(N, H // 2, W // 2, 384, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(128, 64 + 256, generator=g) * 0.05).to(torch.bfloat16).cuda()
    b = torch.randn(128, generator=g).cuda()
    outs = []
    for chunk in (0, 1 << 20):  # one launch; ~1 MB chunks (one 40x40x192 image = 600 KB)
        torch.ops.kvedge.set_conv_chunk_bytes(chunk)
        y = torch.full((N, H, W, 192), 3.0, dtype=torch.bfloat16, device="cuda")
        ops.conv_dual2(skip, 64, low, w, b, ops.ACT_SILU, y, x_coff=128, x2_coff=128, y_coff=64,
                       up2=True)
        outs.append(y.cpu())
    torch.ops.kvedge.set_conv_chunk_bytes(0)
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])
    assert (outs[0][..., :64].float() == 3.0).all()
