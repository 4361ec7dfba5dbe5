"""Numerics of every HIP kernel vs the plain-PyTorch fp32 reference (SURVEY.md §4 T-kernel).

Each test builds inputs on the CPU, runs the reference path (kvedge_amd.ops.reference)
and the gfx950 kernel on the same bf16 inputs, and compares.  The GPU path must be
the native library: tests assert it is loaded (no silent fallback).
"""
import pytest
import torch

from kvedge_amd import ops
from kvedge_amd.ops import ConvSpec

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert ops.load(), "native kvedge library must be loaded on the GPU box"


RRMS_TOL = 4e-3  # rms(err) / rms(ref): ~2-3x the two sides' independent bf16 output rounding


def _rrms(got, ref) -> float:
    """Relative RMS error: a dropped K chunk or a wrong tap moves every element, which
    this sees even when one large output makes the max bound loose."""
    got, ref = got.float(), ref.float()
    return ((got - ref).pow(2).mean().sqrt() / ref.pow(2).mean().sqrt().clamp_min(1e-12)).item()


def _assert_close(got, ref, ctx=None):
    got, ref = got.float(), ref.float()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    rr = _rrms(got, ref)
    assert err <= 0.02 * scale and rr <= RRMS_TOL, (ctx, err, scale, rr)


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(torch.bfloat16)


def _conv_case(N, H, W, cin, cout, k, stride, pad, act, res=False, ldx_extra=0, x_coff=0,
               ldy_extra=0, y_coff=0, tile=-1, seed=0):
    spec = ConvSpec.auto(cin, cout, k, stride, pad, act)
    cin_eff = spec.cin_eff
    ldx = cin_eff + ldx_extra
    x = _rand((N, H, W, ldx), seed)
    if spec.mode == ops.MODE_STEM:
        x[..., 3:] = 0
    g = torch.Generator().manual_seed(seed + 1)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    wp = ops.pack_conv_weight(w, spec)
    Ho, Wo = spec.out_hw(H, W)
    ldy = cout + ldy_extra
    r = _rand((N, Ho, Wo, cout), seed + 2) if res else None
    out_ref = torch.zeros(N, Ho, Wo, ldy, dtype=torch.bfloat16)
    ops.conv2d(x, spec, wp, b, res=r, out=out_ref, x_coff=x_coff, y_coff=y_coff)
    out_gpu = torch.zeros(N, Ho, Wo, ldy, dtype=torch.bfloat16, device="cuda")
    ops.conv2d(x.cuda(), spec, wp.cuda(), b.cuda(), res=None if r is None else r.cuda(),
               out=out_gpu, x_coff=x_coff, y_coff=y_coff, tile=tile)
    torch.cuda.synchronize()
    og = out_gpu.cpu().float()
    orf = out_ref.float()
    err = (og - orf).abs().max().item()
    scale = orf.abs().max().item() + 1e-6
    sl = slice(y_coff, y_coff + cout)
    rr = _rrms(og[..., sl], orf[..., sl])
    assert rr <= RRMS_TOL, ("relative rms", rr)
    # untouched channels outside the output slice must stay zero
    if ldy_extra:
        mask = torch.ones(ldy, dtype=torch.bool)
        mask[y_coff:y_coff + cout] = False
        assert og[..., mask].abs().max().item() == 0.0
    return err, scale


@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, k, stride, pad, act)
    (2, 56, 56, 64, 64, 1, 1, 0, ops.ACT_RELU),      # 1x1 GEMM mode
    (2, 56, 56, 64, 256, 1, 1, 0, ops.ACT_NONE),
    (2, 56, 56, 64, 64, 3, 1, 1, ops.ACT_RELU),      # 3x3 general
    (2, 28, 28, 128, 128, 3, 2, 1, ops.ACT_RELU),    # 3x3 stride 2
    (2, 56, 56, 256, 512, 1, 2, 0, ops.ACT_NONE),    # 1x1 stride-2 downsample
    (1, 7, 7, 512, 512, 3, 1, 1, ops.ACT_RELU),      # tiny spatial tail
    (2, 64, 64, 3, 16, 3, 2, 1, ops.ACT_SILU),       # YOLO stem (stem mode, KW=3)
    (2, 224, 224, 3, 64, 7, 2, 3, ops.ACT_RELU),     # ResNet stem (stem mode, KW=7)
    (2, 20, 20, 48, 32, 1, 1, 0, ops.ACT_SILU),      # Cin not multiple of 64
    (2, 40, 40, 80, 80, 3, 1, 1, ops.ACT_SILU),      # Cin=80 (YOLO cls branch)
    (2, 20, 20, 16, 16, 3, 1, 1, ops.ACT_SILU),      # Cin=16: 4 taps per 64-slab
    (3, 1, 1, 2048, 1000, 1, 1, 0, ops.ACT_NONE),    # FC as GEMM, odd M
])
def test_conv_vs_reference(case):
    err, scale = _conv_case(*case)
    assert err <= 0.02 * scale, (case, err, scale)


def test_conv_residual_and_slices():
    err, scale = _conv_case(2, 28, 28, 64, 128, 3, 1, 1, ops.ACT_RELU, res=True, ldx_extra=64,
                            x_coff=32, ldy_extra=64, y_coff=32)
    assert err <= 0.02 * scale


N_TILES = 121  # v1 (0-5) + v2 (6-31) + v3 (32-53) + v4 (54-57) + v6 (58-67) + v7 BK32 MF16 / direct-epilogue / N-160 (68-85) + v8 split-K (86-104) + v10 (105-107) + v12 (108-116) + v14 (117-120)
PP0 = 117  # v14: 8-phase ping-pong implicit GEMM (conv_pp.hip): 256x256, 512x128, then their
# persistent forms (one workgroup per CU walking tiles); modes 0 (Cin % 64), 1, 4
# + v6 A-resident N-loop 1x1 GEMM (58-67, conv_nloop.hip kNlTiles: one Kpad per tile;
# 63-65 are the fused-downsample (dual) forms, 66-67 step 128 K at a time)
NLOOP0 = 58
XP0 = 68  # v7: the v2 kernel's cross-stage pipelined loop (BK 32 rings, 8 waves)
SK0 = 86  # v8: split-K (conv_sk.hip kSkTiles): K slices per tile (clamped to the K steps)
DE0 = 105  # v10: the direct family's direct-epilogue forms (conv_direct.hip): 8 waves at 1 / 2
# workgroups per CU, the single-patch-buffer 4-wave form at 2 per CU
SKN0 = 108  # v12: skinny edge-batch implicit GEMM (conv_skinny.hip kSknTiles): general /
# 1x1 / dual convs whose every K source has Cin % 64 == 0, M < 65536
# (cin, cout, k, stride, act) instantiated as v10 tile 0 / 1 / 2 (no residual, no fallback)
DE_SHAPES = {
    0: {(64, 64, 3, 1, ops.ACT_RELU), (64, 128, 3, 1, ops.ACT_SILU), (64, 16, 3, 1, ops.ACT_SILU),
        (64, 80, 3, 1, ops.ACT_SILU),
        (64, 64, 3, 1, ops.ACT_SILU), (80, 80, 3, 1, ops.ACT_SILU), (64, 128, 3, 2, ops.ACT_SILU),
        (64, 64, 3, 2, ops.ACT_SILU), (32, 64, 3, 2, ops.ACT_SILU), (16, 32, 3, 2, ops.ACT_SILU),
        (32, 32, 3, 1, ops.ACT_SILU), (16, 16, 3, 1, ops.ACT_SILU), (32, 32, 1, 1, ops.ACT_SILU),
        (48, 32, 1, 1, ops.ACT_SILU), (64, 64, 1, 1, ops.ACT_SILU), (128, 64, 1, 1, ops.ACT_SILU),
        (192, 64, 1, 1, ops.ACT_SILU), (96, 64, 1, 1, ops.ACT_SILU), (64, 64, 1, 1, ops.ACT_NONE),
        (80, 80, 1, 1, ops.ACT_NONE), (128, 128, 3, 1, ops.ACT_RELU), (128, 128, 3, 1, ops.ACT_SILU),
        (128, 128, 3, 2, ops.ACT_SILU)},
    1: {(16, 32, 3, 2, ops.ACT_SILU), (16, 16, 3, 1, ops.ACT_SILU), (32, 64, 3, 2, ops.ACT_SILU),
        (32, 32, 3, 1, ops.ACT_SILU), (32, 32, 1, 1, ops.ACT_SILU), (48, 32, 1, 1, ops.ACT_SILU)},
    2: {(64, 64, 3, 1, ops.ACT_RELU), (64, 128, 3, 1, ops.ACT_SILU), (64, 16, 3, 1, ops.ACT_SILU),
        (64, 80, 3, 1, ops.ACT_SILU), (64, 64, 3, 1, ops.ACT_SILU), (64, 128, 3, 2, ops.ACT_SILU), (64, 64, 3, 2, ops.ACT_SILU),
        (32, 64, 3, 2, ops.ACT_SILU), (32, 32, 3, 1, ops.ACT_SILU), (80, 80, 3, 1, ops.ACT_SILU)},
}


# ... with the residual added after the activation (YOLO C2f bottleneck cv2), tiles 0 / 1
DE_RES_SHAPES = {
    0: {(16, 16, 3, 1, ops.ACT_SILU), (32, 32, 3, 1, ops.ACT_SILU), (64, 64, 3, 1, ops.ACT_SILU)},
    1: {(16, 16, 3, 1, ops.ACT_SILU), (32, 32, 3, 1, ops.ACT_SILU)},
    2: set(),
}


def _de_takes(tile, cin, cout, k, s, act, res):
    """Mirror of direct_plan() for a v10 tile: an instantiated shape, or a Cout covered by
    instantiated slices (largest first, e.g. 144 = 128 + 16); a residual only for its own
    instantiations (no slicing)."""
    if res:
        return (cin, cout, k, s, act) in DE_RES_SHAPES[tile - DE0]
    shapes = DE_SHAPES[tile - DE0]
    if (cin, cout, k, s, act) in shapes:
        return True
    if cout % 16:
        return False
    done = 0
    while done < cout:
        best = max((c for (ci, c, kk, ss, a) in shapes
                    if (ci, kk, ss, a) == (cin, k, s, act) and c <= cout - done), default=0)
        if best == 0:
            return False
        done += best
    return True
NLOOP_KPAD = [128, 256, 256, 256, 256, 384, 384, 768, 256, 256]
NLOOP_DUAL = {63, 64, 65}
STREAM0 = 32  # v3 tiles take 1x1 stride-1 GEMMs and dual-source convs only
DIRECT0 = 54  # v4 direct 3x3 (conv_direct.hip): its instantiation table only
# v2 8-wave (512-thread) tiles 24-28 (256x256 x2, 256x128, 128x256, 256x128 D3) and the
# v_mfma_f32_16x16x32 forms 29-31 (128x128 4-wave, 256x256 and 256x128 8-wave)
# v3 (bm, bn, ring depth, weight slice resident in LDS) -- conv_stream.hip kStreamTiles
STREAM_TILES = [(64, 64, 4, True), (64, 128, 4, True), (128, 64, 4, True), (64, 64, 6, True),
                (64, 128, 3, True), (64, 64, 4, False), (128, 64, 4, False), (128, 128, 3, False),
                (64, 128, 4, False), (64, 128, 3, True), (64, 64, 4, True), (128, 128, 3, False),
                (128, 128, 3, True), (128, 128, 2, True), (128, 128, 3, True),
                (64, 64, 4, True), (64, 128, 3, True), (128, 128, 3, False),  # MF = 16 forms
                (64, 256, 3, True), (64, 256, 2, True),                       # MF = 16 tails
                (64, 256, 3, True), (64, 256, 2, True)]


def _stream_fits(tile, kpad, res):
    """Mirror of stream_lds_bytes(): resident-weight tiles refuse slices > 160 KiB LDS."""
    bm, bn, d, bres = STREAM_TILES[tile - STREAM0]
    lds = 2 * (d * (bm * 64 + (0 if bres else bn * 64)) + (bn * kpad if bres else 0)
               + bm * (bn + 8))
    return lds <= 160 * 1024


def test_tile_count():
    assert int(torch.ops.kvedge.conv_num_tiles()) == N_TILES


@pytest.mark.parametrize("tile", list(range(N_TILES)))
@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, k, stride, pad, act, res, ldx_extra, x_coff)
    (2, 30, 30, 128, 192, 3, 1, 1, ops.ACT_RELU, True, 0, 0),     # KxK, Cin % 64 == 0
    (2, 17, 17, 64, 128, 1, 1, 0, ops.ACT_NONE, False, 32, 16),   # 1x1 GEMM from a slice
    (2, 23, 23, 256, 64, 1, 2, 0, ops.ACT_NONE, False, 0, 0),     # strided 1x1
    (2, 20, 20, 48, 80, 3, 2, 1, ops.ACT_SILU, False, 0, 0),      # generic gather Cin=48
    (1, 9, 9, 16, 64, 4, 1, 2, ops.ACT_RELU, False, 0, 0),        # s2d-stem-like Cin=16 4x4
    (3, 1, 1, 192, 136, 1, 1, 0, ops.ACT_NONE, False, 0, 0),      # K/N tails (Kpad > K)
])
def test_conv_every_tile(tile, case):
    N, H, W, cin, cout, k, s, p, act, res, lx, xc = case
    if tile >= SKN0:
        if cin % 64 == 0:
            err, scale = _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx,
                                    x_coff=xc, tile=tile)
            assert err <= 0.02 * scale, (tile, case, err, scale)
        else:
            with pytest.raises(RuntimeError):
                _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx, x_coff=xc,
                           tile=tile)
        return
    if tile >= DE0:
        if _de_takes(tile, cin, cout, k, s, act, res) and p == k // 2:
            err, scale = _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx,
                                    x_coff=xc, tile=tile)
            assert err <= 0.02 * scale, (tile, case, err, scale)
        else:
            with pytest.raises(RuntimeError):
                _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx, x_coff=xc,
                           tile=tile)
        return
    if NLOOP0 <= tile < XP0:
        # each v6 tile is compiled for one Kpad (128 / 256 / 384 / 768, 1x1 or dual only):
        # none of these cases is one of them
        with pytest.raises(RuntimeError):
            _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx, x_coff=xc,
                       tile=tile)
        return
    if DIRECT0 <= tile < NLOOP0:
        # the direct family takes only its instantiated shapes; of these cases exactly the
        # 1x1 64 -> 128 from a channel slice is one (two Cout slices of the 64 -> 64 form,
        # every direct tile).  The others must be refused (3x3 + residual before the act, no
        # 3x3 48 -> 80 form, strided 1x1, 4x4, Cout 136 with no activation), never run wrong
        # -- and the accepted one must not be refused
        if (cin, cout, k, s) == (64, 128, 1, 1):
            err, scale = _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx,
                                    x_coff=xc, tile=tile)
            assert err <= 0.02 * scale, (tile, case, err, scale)
        else:
            with pytest.raises(RuntimeError):
                _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx, x_coff=xc,
                           tile=tile)
        return
    if STREAM0 <= tile < DIRECT0 and (k != 1 or s != 1 or not _stream_fits(tile, (cin * k * k + 63) // 64 * 64, res)):
        with pytest.raises(RuntimeError):
            _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx, x_coff=xc,
                       tile=tile)
        return
    err, scale = _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx, x_coff=xc,
                            tile=tile)
    assert err <= 0.02 * scale, (tile, case, err, scale)


@pytest.mark.parametrize("tile", [-1] + list(range(STREAM0, DIRECT0)))
@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, act, res, ldx_extra, x_coff, ldy_extra, y_coff)
    (4, 56, 56, 256, 512, ops.ACT_RELU, True, 0, 0, 0, 0),     # several M tiles per workgroup
    (4, 56, 56, 64, 256, ops.ACT_RELU | ops.RES_AFTER_ACT, True, 0, 0, 0, 0),
    (8, 28, 28, 512, 128, ops.ACT_SILU, False, 64, 64, 32, 16),  # slices in and out
    (3, 7, 7, 2048, 1000, ops.ACT_NONE, False, 0, 0, 0, 0),     # N tail, short M
    (5, 13, 13, 40, 72, ops.ACT_SILU, True, 0, 0, 0, 0),       # Cin % 64, Cout % 64 tails
])
def test_conv_stream_gemm(tile, case):
    """Persistent streaming 1x1 kernel: multi-tile walks, residual prefetch across
    tiles, residual before/after the activation, sliced operands, tails."""
    N, H, W, cin, cout, act, res, lx, xc, ly, yc = case
    if tile >= STREAM0 and not _stream_fits(tile, (cin + 63) // 64 * 64, res):
        with pytest.raises(RuntimeError):
            _conv_case(N, H, W, cin, cout, 1, 1, 0, act, res=res, ldx_extra=lx, x_coff=xc,
                       ldy_extra=ly, y_coff=yc, tile=tile)
        return
    err, scale = _conv_case(N, H, W, cin, cout, 1, 1, 0, act, res=res, ldx_extra=lx, x_coff=xc,
                            ldy_extra=ly, y_coff=yc, tile=tile)
    assert err <= 0.02 * scale, (tile, case, err, scale)


@pytest.mark.parametrize("tile", list(range(NLOOP0, XP0)))
@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, act, res, ldx_extra, x_coff, ldy_extra, y_coff)
    (4, 14, 14, 256, 1024, ops.ACT_RELU, True, 0, 0, 0, 0),     # ResNet stage-3 expand + res
    (2, 28, 28, 128, 512, ops.ACT_RELU, True, 0, 0, 0, 0),      # stage-2 expand + res
    (3, 7, 7, 512, 2048, ops.ACT_RELU, True, 0, 0, 0, 0),       # stage-4 expand, M tail
    (2, 15, 13, 256, 136, ops.ACT_SILU | ops.RES_AFTER_ACT, True, 0, 0, 0, 0),  # N tail
    (2, 9, 11, 200, 320, ops.ACT_SILU, False, 64, 40, 32, 16),  # K tail, slices in and out
    (1, 3, 5, 120, 72, ops.ACT_NONE, False, 0, 0, 0, 0),        # one partial M tile, K 120
])
def test_conv_nloop_gemm(tile, case):
    """v6 A-resident N-loop kernel: the counted-wait schedule across many N tiles (warm-up
    and steady state), residual ring, in-place epilogue, K / M / N tails and slices;
    tiles whose K does not match must refuse."""
    N, H, W, cin, cout, act, res, lx, xc, ly, yc = case
    kpad = (cin + 63) // 64 * 64
    if kpad != NLOOP_KPAD[tile - NLOOP0] or tile in NLOOP_DUAL:
        with pytest.raises(RuntimeError):
            _conv_case(N, H, W, cin, cout, 1, 1, 0, act, res=res, ldx_extra=lx, x_coff=xc,
                       ldy_extra=ly, y_coff=yc, tile=tile)
        return
    err, scale = _conv_case(N, H, W, cin, cout, 1, 1, 0, act, res=res, ldx_extra=lx, x_coff=xc,
                            ldy_extra=ly, y_coff=yc, tile=tile)
    assert err <= 0.02 * scale, (tile, case, err, scale)


def test_conv_identity_asymmetric():
    """A = I-style check with an asymmetric B: catches a transposed C write."""
    spec = ConvSpec.auto(64, 64, 1, 1, 0, ops.ACT_NONE)
    x = torch.zeros(1, 8, 8, 64)
    for p in range(64):
        x.view(64, 64)[p, p] = 1.0
    w = torch.arange(64 * 64, dtype=torch.float32).reshape(64, 64, 1, 1) % 17 - 8
    wp = ops.pack_conv_weight(w, spec)
    out = ops.conv2d(x.to(torch.bfloat16).cuda(), spec, wp.cuda(), None)
    torch.cuda.synchronize()
    # out[pixel p, n] = w[n, p]
    ref = w.view(64, 64).t()
    assert torch.equal(out.cpu().float().view(64, 64), ref)


def test_maxpool_avgpool_softmax():
    x = _rand((2, 112, 112, 64), 3)
    y_ref = ops.maxpool2d(x, 3, 2, 1)
    y = ops.maxpool2d(x.cuda(), 3, 2, 1)
    assert torch.equal(y.cpu(), y_ref)
    for shp in ((3, 7, 7, 2048), (1, 7, 7, 2048), (2, 14, 14, 192), (5, 3, 2, 64)):
        f = _rand(shp, 4)
        a = ops.global_avgpool(f.cuda()).cpu().float()
        ref = f.float().mean((1, 2))
        assert ((a - ref).abs() <= 2.0 ** -8 * ref.abs() + 1e-4).all(), shp  # one bf16 rounding
    # 1000 / 1024 / 8 columns: register-resident row path; 1001 / 2000: the strided loop
    for rows, cols in ((5, 1000), (3, 1024), (2, 8), (4, 1001), (2, 2000)):
        lg = _rand((rows, cols), 5, 3.0)
        lg[0, cols // 3] = lg[0, cols // 2] = lg[0].max() + 1  # tie -> the lower index
        p, am = ops.softmax_rows(lg.cuda())
        pr = torch.softmax(lg.float(), 1)
        assert (p.cpu() - pr).abs().max() < 1e-5, (rows, cols)
        assert torch.equal(am.cpu(), lg.float().argmax(1)), (rows, cols)


def test_sppf_and_upsample():
    C = 32
    buf = torch.zeros(2, 20, 20, 4 * C, dtype=torch.bfloat16)
    buf[..., :C] = _rand((2, 20, 20, C), 6)
    ref = ops.sppf_pool(buf.clone(), C)
    got = ops.sppf_pool(buf.cuda(), C).cpu()
    assert torch.equal(got, ref)
    x = _rand((2, 10, 10, 48), 7)
    out_ref = torch.zeros(2, 20, 20, 64, dtype=torch.bfloat16)
    out = torch.zeros(2, 20, 20, 64, dtype=torch.bfloat16, device="cuda")
    ops.upsample2x(x, out_ref, C=32, x_coff=16, y_coff=8)
    ops.upsample2x(x.cuda(), out, C=32, x_coff=16, y_coff=8)
    assert torch.equal(out.cpu(), out_ref)


@pytest.mark.parametrize("N,H,W,C", [(3, 7, 5, 8), (2, 20, 20, 256), (1, 13, 40, 128)])
def test_upsample_slices_and_canary(N, H, W, C):
    """Non-square / odd sizes, channel slices on both sides; untouched channels of the
    destination (the concat partner's slice) must keep their NaN canary."""
    ldx, ldy = C + 16, C + 24
    x = _rand((N, H, W, ldx), 11)
    out_ref = torch.full((N, 2 * H, 2 * W, ldy), float("nan"), dtype=torch.bfloat16)
    out = out_ref.clone().cuda()
    ops.upsample2x(x, out_ref, C=C, x_coff=8, y_coff=16)
    ops.upsample2x(x.cuda(), out, C=C, x_coff=8, y_coff=16)
    got = out.cpu()
    assert torch.equal(got[..., 16:16 + C], out_ref[..., 16:16 + C])
    assert torch.isnan(got[..., :16]).all() and torch.isnan(got[..., 16 + C:]).all()


def test_synth_preprocess_bn():
    fr = torch.empty(2, 16, 16, 3, dtype=torch.uint8)
    ops.synth_frames(fr, 7, 3)
    frg = torch.empty(2, 16, 16, 3, dtype=torch.uint8, device="cuda")
    ops.synth_frames(frg, 7, 3)
    assert torch.equal(frg.cpu(), fr)
    ctr = torch.tensor([3], dtype=torch.int64, device="cuda")
    ops.synth_frames(frg, 7, ctr)
    assert torch.equal(frg.cpu(), fr) and int(ctr.item()) == 4
    # [counter, done-count] form: the kernel's last block bumps the counter (one launch),
    # many blocks, repeatedly; the done-count slot is re-armed to 0 every time
    big = torch.empty(8, 64, 64, 3, dtype=torch.uint8, device="cuda")
    big_ref = torch.empty(8, 64, 64, 3, dtype=torch.uint8)
    ctr2 = torch.tensor([3, 0], dtype=torch.int64, device="cuda")
    for k in range(5):
        ops.synth_frames(big, 7, ctr2)
        ops.synth_frames(big_ref, 7, 3 + k)
        torch.cuda.synchronize()
        assert torch.equal(big.cpu(), big_ref) and ctr2.tolist() == [4 + k, 0], (k, ctr2.tolist())
    # a grid too large for the in-kernel ticket (2048 blocks): the separate bump launch
    huge = torch.empty(48, 224, 224, 3, dtype=torch.uint8, device="cuda")
    ctr3 = torch.tensor([9, 0], dtype=torch.int64, device="cuda")
    ops.synth_frames(huge, 7, ctr3)
    ops.synth_frames(huge, 7, ctr3)
    torch.cuda.synchronize()
    assert ctr3.tolist() == [11, 0]
    ref2 = torch.empty(2, 224, 224, 3, dtype=torch.uint8)
    ops.synth_frames(ref2, 7, 10)
    assert torch.equal(huge[:2].cpu(), ref2)
    p_ref = ops.preprocess(fr)
    p = ops.preprocess(fr.cuda()).cpu()
    assert (p.float() - p_ref.float()).abs().max() <= 0.02
    x = _rand((4, 5, 5, 64), 8)
    sc = torch.rand(64) + 0.5
    sh = torch.randn(64)
    y_ref = ops.batchnorm_nhwc(x, sc, sh, relu=True)
    y = ops.batchnorm_nhwc(x.cuda(), sc.cuda(), sh.cuda(), relu=True).cpu()
    assert (y.float() - y_ref.float()).abs().max() <= 0.05


@pytest.mark.parametrize("hs,nc", [((16, 8, 4), 80), ((10, 5, 3), 80), ((12, 6, 3), 16),
                                   (((24, 40), (12, 20), (6, 10)), 80),
                                   (((9, 13), (5, 7), (3, 4)), 8)])
def test_yolo_decode_and_nms(hs, nc):
    """nc = 80 runs the compile-time class-count instantiation, others the generic one;
    non-square levels exercise the float-reciprocal anchor row/col split."""
    hw = [h if isinstance(h, tuple) else (h, h) for h in hs]
    feats = [_rand((2, h, w, 64 + nc), 10 + i, 2.0) for i, (h, w) in enumerate(hw)]
    b_ref, s_ref, c_ref = ops.yolo_decode(feats, (8, 16, 32), nc)
    b, s, c = ops.yolo_decode([f.cuda() for f in feats], (8, 16, 32), nc)
    assert (b.cpu() - b_ref).abs().max() < 2e-2
    assert (s.cpu() - s_ref).abs().max() < 1e-5
    assert torch.equal(c.cpu(), c_ref)
    out_ref, cnt_ref = ops.nms(b_ref, s_ref, c_ref, conf=0.6, iou=0.5, max_det=100)
    out, cnt = ops.nms(b_ref.cuda(), s_ref.cuda(), c_ref.cuda(), conf=0.6, iou=0.5, max_det=100)
    assert torch.equal(cnt.cpu(), cnt_ref)
    assert (out.cpu() - out_ref).abs().max() < 1e-4


def test_nms_dense_overlaps():
    """Many heavily-overlapping boxes of few classes: exercises in-chunk suppression."""
    g = torch.Generator().manual_seed(11)
    A = 700
    ctr = torch.rand(1, A, 2, generator=g) * 100
    wh = torch.rand(1, A, 2, generator=g) * 30 + 5
    boxes = torch.cat([ctr - wh / 2, ctr + wh / 2], -1)
    scores = torch.rand(1, A, generator=g)
    cls = torch.randint(0, 3, (1, A), generator=g, dtype=torch.int32)
    o_ref, n_ref = ops.nms(boxes, scores, cls, conf=0.1, iou=0.45, max_det=300)
    o, n = ops.nms(boxes.cuda(), scores.cuda(), cls.cuda(), conf=0.1, iou=0.45, max_det=300)
    assert torch.equal(n.cpu(), n_ref)
    assert (o.cpu() - o_ref).abs().max() < 1e-4


@pytest.mark.parametrize("bucket", [False, True])
@pytest.mark.parametrize("case", ["spread", "clustered", "ties", "piles"])
def test_nms_top_set(case, bucket, monkeypatch):
    """YOLO-sized candidate lists (8400 anchors, most above conf) through the NMS top-set
    path: 'spread' reaches max_det inside the bucket-sorted top set; 'clustered' (one class,
    boxes piled on few centres) exhausts the top set first and falls back to the full sort;
    'ties' (scores on 8 levels) puts > 2048 keys in one histogram bin (full-sort path);
    'piles' (scores on 96 levels) keeps the top set under 2048 keys but puts > 64 in a bin
    (the bucket sort's bitonic fallback).  bucket: the opt-in histogram bucket sort of the
    top set (KVEDGE_NMS_DIAG bit 3) instead of the default bitonic network."""
    if bucket:
        monkeypatch.setenv("KVEDGE_NMS_DIAG", "8")
    g = torch.Generator().manual_seed(5)
    A, N = 8400, 3
    if case == "clustered":
        ctr = torch.rand(N, 4, 2, generator=g)[:, torch.randint(0, 4, (A,), generator=g)] * 600
        wh = torch.rand(N, A, 2, generator=g) * 4 + 60
        cls = torch.zeros(N, A, dtype=torch.int32)
    else:
        ctr = torch.rand(N, A, 2, generator=g) * 640
        wh = torch.rand(N, A, 2, generator=g) * 40 + 4
        cls = torch.randint(0, 80, (N, A), generator=g, dtype=torch.int32)
    boxes = torch.cat([ctr - wh / 2, ctr + wh / 2], -1)
    scores = torch.rand(N, A, generator=g) * 0.7 + 0.3
    if case == "ties":
        scores = (scores * 8).floor() / 8 + 0.05
    if case == "piles":
        scores = (scores * 96).floor() / 96 + 0.002
    o_ref, n_ref = ops.nms(boxes, scores, cls, conf=0.25, iou=0.7, max_det=300)
    o, n = ops.nms(boxes.cuda(), scores.cuda(), cls.cuda(), conf=0.25, iou=0.7, max_det=300)
    assert torch.equal(n.cpu(), n_ref), (n, n_ref)
    assert (o.cpu() - o_ref).abs().max() < 1e-4
    if case == "clustered":
        assert int(n_ref.max()) < 300  # the top set alone never reaches max_det here


@pytest.mark.parametrize("tile", [-1] + list(range(6, DIRECT0)) + sorted(NLOOP_DUAL) + [NLOOP0 + 8]
                         + list(range(XP0, N_TILES)))
@pytest.mark.parametrize("geom", [(2, 14, 14, 64, 128, 256, 2), (2, 7, 7, 128, 256, 512, 1),
                                  (1, 5, 5, 64, 64, 128, 2),
                                  # the v6 dual tiles' K: 128 + 256 and 256 + 512, tails
                                  (2, 14, 13, 128, 256, 512, 2), (1, 5, 5, 128, 256, 136, 1),
                                  (2, 7, 9, 256, 512, 1024, 2)])
def test_conv_dual_fused_downsample(tile, geom):
    N, Ho, Wo, K1, K2, cout, s = geom
    g = torch.Generator().manual_seed(tile + 5)
    x1 = torch.randn(N, Ho, Wo, K1, generator=g).to(torch.bfloat16)
    x2 = torch.randn(N, Ho * s, Wo * s, K2, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, K1 + K2, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(cout, generator=g)
    ref = ops.conv_dual(x1, x2, w, b, ops.ACT_RELU, s)
    if DE0 <= tile < SKN0:
        with pytest.raises(RuntimeError):  # the v10 direct forms take no dual-source GEMM
            ops.conv_dual(x1.cuda(), x2.cuda(), w.cuda(), b.cuda(), ops.ACT_RELU, s, tile=tile)
        return
    if NLOOP0 <= tile < XP0 and (tile not in NLOOP_DUAL or K1 + K2 != NLOOP_KPAD[tile - NLOOP0]):
        with pytest.raises(RuntimeError):  # each v6 dual tile is compiled for one K
            ops.conv_dual(x1.cuda(), x2.cuda(), w.cuda(), b.cuda(), ops.ACT_RELU, s, tile=tile)
        return
    if STREAM0 <= tile < DIRECT0 and not _stream_fits(tile, K1 + K2, False):
        with pytest.raises(RuntimeError):  # resident weight slice exceeds 160 KiB of LDS
            ops.conv_dual(x1.cuda(), x2.cuda(), w.cuda(), b.cuda(), ops.ACT_RELU, s, tile=tile)
        return
    got = ops.conv_dual(x1.cuda(), x2.cuda(), w.cuda(), b.cuda(), ops.ACT_RELU, s, tile=tile)
    torch.cuda.synchronize()
    _assert_close(got.cpu(), ref, ("dual", tile, geom))


def test_conv_dual_rejects_v1_tiles():
    x1 = torch.zeros(1, 4, 4, 64, dtype=torch.bfloat16, device="cuda")
    x2 = torch.zeros(1, 4, 4, 64, dtype=torch.bfloat16, device="cuda")
    w = torch.zeros(64, 128, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(RuntimeError):
        ops.conv_dual(x1, x2, w, None, ops.ACT_NONE, 1, tile=0)


@pytest.mark.parametrize("tile", [-1, 1, 6, 7, 12, 13, STREAM0, STREAM0 + 1, STREAM0 + 5, DIRECT0,
                                  DIRECT0 + 1, XP0, XP0 + 4, SK0, SK0 + 9, DE0, DE0 + 2,
                                  SKN0, SKN0 + 4, SKN0 + 6, SKN0 + 8])
@pytest.mark.parametrize("k", [1, 3])
def test_conv_poisoned_canary(tile, k):
    """SURVEY §5.2 poisoned-buffer check: the output buffer is NaN-filled, with a NaN
    canary tail after the tensor and NaN in the channels outside the written slice.  Every
    written element must be finite, and every byte outside the slice must stay NaN
    (a kernel that writes past M/N tails or outside [y_coff, y_coff+cout) fails here)."""
    if STREAM0 <= tile < DIRECT0 and k != 1:
        pytest.skip("v3 tiles take 1x1 GEMMs only")
    if (DIRECT0 <= tile < XP0 or DE0 <= tile < SKN0) and k != 3:
        pytest.skip("v4 / v10 take 3x3 only here")
    N, H, W, cin, cout, ldy, y_coff = 3, 13, 11, 64, 72, 104, 16
    if DIRECT0 <= tile < XP0 or DE0 <= tile < SKN0:
        cout = 64  # an instantiated direct shape (64 -> 64 ReLU)
    spec = ConvSpec.auto(cin, cout, k, 1, k // 2, ops.ACT_RELU)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, H, W, cin, generator=g).to(torch.bfloat16).cuda()
    w = ops.pack_conv_weight(torch.randn(cout, cin, k, k, generator=g) * 0.1, spec).cuda()
    b = torch.randn(cout, generator=g).cuda()
    Ho, Wo = spec.out_hw(H, W)
    n_out = N * Ho * Wo * ldy
    flat = torch.full((n_out + 4096,), float("nan"), dtype=torch.bfloat16, device="cuda")
    out = flat[:n_out].view(N, Ho, Wo, ldy)
    ops.conv2d(x, spec, w, b, out=out, y_coff=y_coff, tile=tile)
    torch.cuda.synchronize()
    o = out.cpu().float()
    inside = o[..., y_coff:y_coff + cout]
    assert torch.isfinite(inside).all()
    mask = torch.ones(ldy, dtype=torch.bool)
    mask[y_coff:y_coff + cout] = False
    assert torch.isnan(o[..., mask]).all()
    assert torch.isnan(flat[n_out:].cpu().float()).all()
    ref = ops.conv2d(x.cpu(), spec, w.cpu(), b.cpu())
    _assert_close(inside, ref, ("canary", tile, k))


@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, stride, act, res, ldx_extra, x_coff, ldy_extra, y_coff)
    (2, 56, 56, 64, 64, 1, ops.ACT_RELU, False, 0, 0, 0, 0),     # ResNet-50 layer1 conv2
    (3, 13, 11, 64, 64, 1, ops.ACT_RELU, False, 0, 0, 0, 0),     # H % 4, pixel-block tails
    (1, 1, 1, 64, 64, 1, ops.ACT_NONE, False, 0, 0, 0, 0),
    (2, 9, 62, 64, 64, 1, ops.ACT_SILU, True, 64, 64, 32, 16),   # widest row, slices, +res
    (2, 40, 40, 16, 32, 2, ops.ACT_SILU, False, 0, 0, 0, 0),     # YOLO b1 (stride 2)
    (2, 21, 19, 16, 16, 1, ops.ACT_SILU, True, 16, 16, 16, 0),   # C2f bottleneck 16
    (2, 20, 20, 32, 64, 2, ops.ACT_SILU, False, 0, 0, 0, 0),     # YOLO b3
    (2, 20, 20, 32, 32, 1, ops.ACT_SILU, True, 0, 0, 0, 0),
    (2, 40, 40, 64, 64, 1, ops.ACT_SILU, True, 0, 0, 0, 0),      # C2f bottleneck 64 (+res)
    (3, 13, 11, 32, 32, 1, ops.ACT_SILU, True, 32, 32, 8, 8),    # +res: tails, x / y slices
    (2, 19, 17, 64, 128, 2, ops.ACT_SILU, False, 0, 0, 0, 0),    # YOLO b5 (odd H, W)
    (2, 10, 10, 64, 64, 2, ops.ACT_SILU, False, 0, 0, 0, 0),     # h16
    (1, 160, 160, 16, 16, 1, ops.ACT_SILU, False, 0, 0, 0, 0),   # full YOLO row width
    (2, 20, 20, 64, 144, 1, ops.ACT_SILU, False, 0, 0, 16, 8),   # Detect stem: 128 + 16 split
    (2, 23, 21, 64, 80, 1, ops.ACT_SILU, False, 0, 0, 8, 8),     # its 80-wide slice alone
    (2, 80, 80, 80, 80, 1, ops.ACT_SILU, False, 64, 64, 0, 0),   # Detect P3 cls 3x3 (NCB = 3)
    (3, 13, 11, 80, 80, 1, ops.ACT_SILU, False, 0, 0, 8, 8),     # pixel-block tails, y slice
    (2, 40, 40, 80, 80, 1, ops.ACT_SILU, False, 64, 64, 0, 0),   # Detect P4 cls
    (3, 28, 28, 128, 128, 1, ops.ACT_RELU, False, 0, 0, 0, 0),   # ResNet stage-2 conv2 (4 waves)
    (2, 13, 11, 128, 128, 1, ops.ACT_RELU, False, 0, 0, 8, 8),   # band / pixel-block tails
    (2, 20, 20, 128, 128, 1, ops.ACT_SILU, False, 0, 0, 0, 0),   # YOLO P5 3x3 (v10 only)
    (2, 41, 39, 128, 128, 2, ops.ACT_SILU, False, 0, 0, 8, 8),   # YOLO PAN downsample (v10 only)
])
@pytest.mark.parametrize("dtile", [0, 1, 3, "de0", "de1", "de2"])
def test_conv_direct3x3(case, dtile):
    """v4 persistent direct 3x3 conv (csrc/kernels/conv_direct.hip) vs the fp32 reference:
    both strides, odd sizes, channel slices in/out, residual after the activation.
    dtile 0: VGPR-prefetched band patch; 1: the DMA (buffer_load ... lds) double buffer;
    3: the DMA form at two workgroups per CU (narrow shapes; others fall back to 0/1);
    de0 / de1: the v10 direct-epilogue forms (accumulators straight to HBM), which refuse
    every shape they do not instantiate."""
    N, H, W, cin, cout, s, act, res, lx, xc, ly, yc = case
    a = act | (ops.RES_AFTER_ACT if res and act != ops.ACT_NONE else 0)
    tile = DE0 + int(dtile[2]) if isinstance(dtile, str) else DIRECT0 + dtile
    v10_only = (cin, cout, s, act) in {(128, 128, 1, ops.ACT_SILU), (128, 128, 2, ops.ACT_SILU)}
    if (tile >= DE0 and not _de_takes(tile, cin, cout, 3, s, act, res)) or (tile < DE0 and v10_only):
        with pytest.raises(RuntimeError):
            _conv_case(N, H, W, cin, cout, 3, s, 1, a, res=res, ldx_extra=lx, x_coff=xc,
                       ldy_extra=ly, y_coff=yc, tile=tile)
        return
    err, scale = _conv_case(N, H, W, cin, cout, 3, s, 1, a, res=res, ldx_extra=lx, x_coff=xc,
                            ldy_extra=ly, y_coff=yc, tile=tile)
    assert err <= 0.02 * scale, (case, err, scale)


@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, act, ldx_extra, x_coff, ldy_extra, y_coff) -- YOLO's 1x1 convs
    (2, 160, 160, 32, 32, ops.ACT_SILU, 0, 0, 16, 0),    # C2f b2 cv1 into the 48-ch buffer
    (2, 160, 160, 48, 32, ops.ACT_SILU, 0, 0, 0, 0),     # C2f b2 cv2
    (2, 80, 80, 64, 64, ops.ACT_SILU, 0, 0, 64, 0),
    (2, 80, 80, 128, 64, ops.ACT_SILU, 0, 0, 128, 64),
    (2, 80, 80, 192, 64, ops.ACT_SILU, 0, 0, 32, 32),
    (2, 80, 80, 96, 64, ops.ACT_SILU, 32, 16, 0, 0),     # input channel slice
    (2, 80, 80, 64, 64, ops.ACT_NONE, 0, 0, 80, 0),      # Detect box 1x1 into the head map
    (2, 80, 80, 80, 80, ops.ACT_NONE, 0, 0, 64, 64),     # Detect cls 1x1 (NCB = 3)
    (3, 13, 11, 32, 32, ops.ACT_SILU, 0, 0, 0, 0),       # pixel-block / band tails
    (1, 1, 1, 48, 32, ops.ACT_SILU, 0, 0, 0, 0),
])
@pytest.mark.parametrize("dtile", [0, 1, 3, "de0", "de1", "de2"])
def test_conv_direct1x1(case, dtile):
    """v4 direct family in its 1x1 form (KK = 1, pad 0) vs the fp32 reference: channel
    slices in and out, tails, both patch-fetch forms, the v10 direct-epilogue forms."""
    N, H, W, cin, cout, act, lx, xc, ly, yc = case
    tile = DE0 + int(dtile[2]) if isinstance(dtile, str) else DIRECT0 + dtile
    if tile >= DE0 and not _de_takes(tile, cin, cout, 1, 1, act, False):
        with pytest.raises(RuntimeError):
            _conv_case(N, H, W, cin, cout, 1, 1, 0, act, ldx_extra=lx, x_coff=xc,
                       ldy_extra=ly, y_coff=yc, tile=tile)
        return
    err, scale = _conv_case(N, H, W, cin, cout, 1, 1, 0, act, ldx_extra=lx, x_coff=xc,
                            ldy_extra=ly, y_coff=yc, tile=tile)
    assert err <= 0.02 * scale, (case, err, scale)


@pytest.mark.parametrize("shape", [(2, 40, 40), (1, 13, 7)])
def test_conv_direct_s2d_stem(shape):
    """v4 in its 2x2 form: the space-to-depth YOLO stem (stride-2 3x3 on RGB as a stride-1
    2x2 over [N,H/2,W/2,16] with top/left pad 1, bottom/right pad 0), SiLU."""
    N, H, W = shape
    spec = ConvSpec(16, 16, 2, 2, 1, 1, ops.ACT_SILU, ops.MODE_GENERAL, pad_b=0)
    x = _rand((N, H, W, 16), 11)
    g = torch.Generator().manual_seed(12)
    wp = ops.pack_conv_weight(torch.randn(16, 16, 2, 2, generator=g) * 0.2, spec)
    b = torch.randn(16, generator=g) * 0.1
    ref = ops.conv2d(x, spec, wp, b)
    got = ops.conv2d(x.cuda(), spec, wp.cuda(), b.cuda(), tile=DIRECT0)
    torch.cuda.synchronize()
    assert got.shape == ref.shape == (N, H, W, 16)
    _assert_close(got.cpu(), ref, ("s2d stem", shape))


def test_conv_direct3x3_rejects():
    with pytest.raises(RuntimeError):  # W + 2 patch wider than the prefetch budget allows
        _conv_case(1, 4, 1200, 64, 64, 3, 1, 1, ops.ACT_RELU, tile=DIRECT0)
    with pytest.raises(RuntimeError):  # not instantiated
        _conv_case(1, 8, 8, 48, 48, 3, 1, 1, ops.ACT_RELU, tile=DIRECT0)


@pytest.mark.parametrize("shape", [(2, 112, 112), (3, 17, 13), (1, 8, 30), (20, 112, 112),
                                   (120, 17, 13), (300, 6, 8)])
def test_stem_pool_fused(shape):
    """Fused s2d stem conv + ReLU + 3x3/2 max pool == reference conv then reference pool.
    More bands than CUs (the last three shapes) make every workgroup walk several bands,
    reusing the shared stem row from its 5-row tile ring, with ranges that cross image
    boundaries (odd H: a last band whose lower stem rows are outside the image)."""
    from kvedge_amd.models.layers import DeployedConv
    import torch.nn as nn
    N, H, W = shape
    torch.manual_seed(5)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
    bn = nn.BatchNorm2d(64).eval()
    bn.running_mean.uniform_(-0.2, 0.2)
    bn.running_var.uniform_(0.5, 1.5)
    stem = DeployedConv.stem_s2d(conv, bn, ops.ACT_RELU)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(N, H, W, 16, generator=g).to(torch.bfloat16)
    x[..., 3::4] = 0  # the s2d layout's pad channel
    ref = ops.stem_pool(x, stem.spec, stem.w, stem.b)
    out = torch.full((N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, 72), float("nan"),
                     dtype=torch.bfloat16, device="cuda")
    ops.stem_pool(x.cuda(), stem.spec, stem.w.cuda(), stem.b.cuda(), out=out, y_coff=8)
    torch.cuda.synchronize()
    got = out.cpu().float()
    assert torch.isnan(got[..., :8]).all()
    _assert_close(got[..., 8:], ref, ("stem_pool", shape))


@pytest.mark.parametrize("case", [
    # (N, H, W, k1, k2 (0 = plain conv3 + residual), stride2, n_t)
    (2, 56, 56, 64, 0, 1, 64),     # layer1 conv3 + res -> next conv1 (64)
    (2, 56, 56, 64, 0, 1, 128),    # layer1 -> layer2 conv1 (128)
    (3, 13, 11, 64, 0, 1, 64),     # M tail (M % 64 != 0)
    (12, 56, 56, 64, 0, 1, 64),    # more 64-row tiles than CUs: workgroups walk several tiles
    (2, 28, 28, 64, 64, 1, 64),    # fused downsample dual form (layer1 block 0)
    (1, 9, 7, 64, 64, 2, 64),      # dual with a strided second source
])
@pytest.mark.parametrize("mf", [32, 16])
def test_conv_tail_fused(case, mf):
    """v3 fused bottleneck tail: y = ReLU(t . W3 (+ x . Wd) + b (+ res)) and the next
    block's conv1 z = ReLU(y . W1 + b1) in one kernel, vs the reference composition."""
    N, H, W, k1, k2, s2, nt = case
    cout = 256
    # default tile = the 32x32x16 tail of this n_t; the v_mfma_f32_16x16x32 tails sit 2 before
    tile = -1 if mf == 32 else DIRECT0 - (4 if nt == 64 else 3)
    g = torch.Generator().manual_seed(nt + k2 + H)
    t = _rand((N, H, W, k1), 1)
    w = (torch.randn(cout, k1 + k2, generator=g) * (2.0 / (k1 + k2)) ** 0.5).to(torch.bfloat16)
    b = torch.randn(cout, generator=g) * 0.1
    w1 = (torch.randn(nt, cout, generator=g) * (2.0 / cout) ** 0.5).to(torch.bfloat16)
    b1 = torch.randn(nt, generator=g) * 0.1
    if k2:
        x2 = _rand((N, H * s2, W * s2, k2), 2)
        y_ref, z_ref = ops.conv_tail(t, w, b, ops.ACT_RELU, w1, b1, x2=x2, stride2=s2)
        y, z = ops.conv_tail(t.cuda(), w.cuda(), b.cuda(), ops.ACT_RELU, w1.cuda(), b1.cuda(),
                             x2=x2.cuda(), stride2=s2, tile=tile)
    else:
        r = _rand((N, H, W, cout), 3)
        y_ref, z_ref = ops.conv_tail(t, w, b, ops.ACT_RELU, w1, b1, res=r)
        y, z = ops.conv_tail(t.cuda(), w.cuda(), b.cuda(), ops.ACT_RELU, w1.cuda(), b1.cuda(),
                             res=r.cuda(), tile=tile)
    torch.cuda.synchronize()
    for got, ref in ((y, y_ref), (z, z_ref)):
        _assert_close(got.cpu(), ref, ("tail", case, mf))



@pytest.mark.parametrize("tile", list(range(SK0, DE0)))
@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, k, stride, act, res) -- ResNet-50 edge-batch shapes
    (1, 14, 14, 256, 256, 3, 1, ops.ACT_RELU, False),     # s3 3x3 at batch 1: M 196
    (1, 7, 7, 512, 512, 3, 1, ops.ACT_RELU, False),       # s4 3x3: M 49, K 4608
    (1, 7, 7, 512, 2048, 1, 1, ops.ACT_RELU, True),       # s4 conv3 + residual
    (2, 14, 14, 1024, 256, 1, 1, ops.ACT_RELU, False),    # s3 conv1, M tail
    (1, 14, 14, 512, 512, 3, 2, ops.ACT_RELU, False),     # s4 block-0 3x3 / 2
])
def test_conv_splitk(tile, case):
    """v8 split-K: each K slice writes its fp32 partial tile to its own slab of the stream's
    workspace (plain stores), the finalize kernel sums the slabs and applies bias / residual
    / activation.  The workspace is poisoned with NaN first: no output may depend on its old
    contents (every slab element the finalize reads is written by its slice)."""
    N, H, W, cin, cout, k, s, act, res = case
    Ho, Wo = (H + 2 * (k // 2) - k) // s + 1, (W + 2 * (k // 2) - k) // s + 1
    ws = ops.splitk_workspace(torch.device("cuda", torch.cuda.current_device()), N * Ho * Wo * cout)
    assert ws is not None
    ws.fill_(float("nan"))
    err, scale = _conv_case(N, H, W, cin, cout, k, s, k // 2, act, res=res, tile=tile)
    assert err <= 0.02 * scale, (tile, case, err, scale)


@pytest.mark.parametrize("tile", [0, 1])
@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, c2, ldx, x_coff, ldz, z_coff) -- YOLOv8n Detect branch pairs
    (2, 80, 80, 64, 64, 64, 144, 0, 144, 0),     # P3 box branch (s[:, :64]) -> head[:, :64]
    (2, 80, 80, 80, 80, 80, 144, 64, 144, 64),   # P3 cls branch (s[:, 64:]) -> head[:, 64:]
    (3, 40, 40, 64, 64, 64, 144, 0, 144, 0),     # P4
    (3, 20, 20, 80, 80, 80, 144, 64, 144, 64),   # P5
    (2, 13, 7, 64, 64, 64, 64, 0, 80, 8),        # odd geometry, band tails
])
def test_conv_pair(tile, case):
    """Fused Detect-branch pair (ops.conv_pair: 3x3 + SiLU, then 1x1 + bias from the LDS
    output tile) vs the two reference convs with the bf16 intermediate; NaN canaries around
    the head-map slice it writes."""
    N, H, W, cin, cout, c2, ldx, xo, ldz, zo = case
    spec = ConvSpec.auto(cin, cout, 3, 1, 1, ops.ACT_SILU)
    g = torch.Generator().manual_seed(cin + H)
    x = _rand((N, H, W, ldx), 11)
    w = ops.pack_conv_weight(torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cin)) ** 0.5, spec)
    b = torch.randn(cout, generator=g) * 0.1
    w2 = (torch.randn(c2, cout, generator=g) * (1.0 / cout) ** 0.5).to(torch.bfloat16)
    b2 = torch.randn(c2, generator=g) * 0.1
    ref = torch.zeros(N, H, W, ldz, dtype=torch.bfloat16)
    ops.conv_pair(x, spec, w, b, w2, b2, ref, x_coff=xo, z_coff=zo)
    out = torch.full((N, H, W, ldz), float("nan"), dtype=torch.bfloat16, device="cuda")
    ops.conv_pair(x.cuda(), spec, w.cuda(), b.cuda(), w2.cuda(), b2.cuda(), out, x_coff=xo,
                  z_coff=zo, tile=tile)
    torch.cuda.synchronize()
    got = out.cpu()
    assert torch.isnan(got[..., :zo].float()).all() and torch.isnan(got[..., zo + c2:].float()).all()
    _assert_close(got[..., zo:zo + c2], ref[..., zo:zo + c2], ("pair", case, tile))


@pytest.mark.parametrize("N,H,W,C,ncls,ldw", [(1, 7, 7, 2048, 1000, 2048), (5, 7, 7, 2048, 1000, 2048),
                                              (3, 3, 5, 64, 40, 128), (16, 7, 7, 2048, 1000, 2048)])
def test_pooled_fc(N, H, W, C, ncls, ldw):
    """Edge-batch classifier head (avgpool + fc in one GEMV launch) vs the two reference ops
    (bf16 pooled vector in between); Kpad > C exercises the weight row pitch."""
    x = _rand((N, H, W, C), 21)
    g = torch.Generator().manual_seed(C + ncls)
    w = (torch.randn(ncls, ldw, generator=g) * (1.0 / C) ** 0.5).to(torch.bfloat16)
    b = torch.randn(ncls, generator=g) * 0.1
    ref = ops.pooled_fc(x, w, b)
    got = ops.pooled_fc(x.cuda(), w.cuda(), b.cuda())
    torch.cuda.synchronize()
    assert got.shape == ref.shape == (N, ncls)
    _assert_close(got.cpu(), ref, ("pooled_fc", N, C, ncls))


def _seam_tiles():
    try:
        return int(torch.ops.kvedge.conv_seam_num_tiles()) if ops.load() else 0
    except Exception:  # noqa: BLE001 -- collection on a box without the library
        return 0


@pytest.mark.parametrize("case", [
    # (N, H, W, k3, n_t) -- conv3 K3 -> Cout = 4 K3 (+ residual) -> next conv1 n_t
    (2, 28, 28, 128, 128),    # stage-2 seam
    (3, 13, 11, 128, 128),    # M tail (M % 128 != 0)
    (2, 28, 28, 128, 256),    # stage 2 -> 3 boundary
    (2, 14, 14, 256, 256),    # stage-3 seam
    (1, 9, 7, 256, 256),      # one partial row block
    (2, 14, 14, 256, 512),    # stage 3 -> 4 boundary
])
def test_conv_seam(case):
    """v9 seam (conv_seam.hip): y = ReLU(t . W3^T + b3 + res) and z = ReLU(y . W1^T + b1) in
    one kernel, vs the reference composition (bf16 y in between), through every seam tile
    that takes the shape; y and z outputs NaN-poisoned first."""
    N, H, W, k3, nt = case
    cout = 4 * k3
    g = torch.Generator().manual_seed(k3 + nt + H)
    t = _rand((N, H, W, k3), 5)
    w = (torch.randn(cout, k3, generator=g) * (2.0 / k3) ** 0.5).to(torch.bfloat16)
    b = torch.randn(cout, generator=g) * 0.1
    w1 = (torch.randn(nt, cout, generator=g) * (2.0 / cout) ** 0.5).to(torch.bfloat16)
    b1 = torch.randn(nt, generator=g) * 0.1
    r = _rand((N, H, W, cout), 6)
    y_ref, z_ref = ops.conv_tail(t, w, b, ops.ACT_RELU, w1, b1, res=r)
    base = int(torch.ops.kvedge.conv_num_tiles())
    ran = 0
    for st in [-1] + list(range(_seam_tiles())):
        y = torch.full((N, H, W, cout), float("nan"), dtype=torch.bfloat16, device="cuda")
        z = torch.full((N, H, W, nt), float("nan"), dtype=torch.bfloat16, device="cuda")
        try:
            ops.conv_tail(t.cuda(), w.cuda(), b.cuda(), ops.ACT_RELU, w1.cuda(), b1.cuda(),
                          res=r.cuda(), out=y, z=z, tile=-1 if st < 0 else base + st)
        except RuntimeError as e:
            assert st >= 0 and ("rc=-8" in str(e) or "rc=-11" in str(e)), (st, e)
            continue  # that tile's K3 / n_t differ from the shape
        torch.cuda.synchronize()
        ran += 1
        for got, ref in ((y, y_ref), (z, z_ref)):
            assert not torch.isnan(got.float()).any(), ("seam nan", case, st)
            _assert_close(got.cpu(), ref, ("seam", case, st))
    assert ran >= 2, "the default pick and at least one explicit seam tile must run"


@pytest.mark.parametrize("tile", list(range(SKN0, N_TILES)))
@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, k, stride, pad, act, res): ResNet-50 edge-batch layers
    (1, 14, 14, 256, 256, 3, 1, 1, ops.ACT_RELU, False),    # stage-3 3x3 (36 chunks)
    (1, 14, 14, 512, 512, 3, 2, 1, ops.ACT_RELU, False),    # stage-4 entry 3x3/2 (72 chunks)
    (1, 7, 7, 2048, 512, 1, 1, 0, ops.ACT_RELU, False),     # stage-4 reduce (M = 49 tail)
    (3, 7, 7, 512, 2048, 1, 1, 0, ops.ACT_RELU, True),      # stage-4 expand + residual
    (1, 1, 1, 2048, 1000, 1, 1, 0, ops.ACT_NONE, False),    # FC: M = 1, Cout tail
    (2, 28, 28, 128, 128, 3, 1, 1, ops.ACT_RELU, False),    # stage 2 at b2 (M = 1568)
])
def test_skinny_edge_shapes(tile, case):
    """v12 (conv_skinny.hip) at the layer shapes it is for: multi-pass K (every tile's
    per-pass reach is below the 4608-deep stage-4 3x3), padding taps, M and Cout tails."""
    N, H, W, cin, cout, k, s, p, act, res = case
    err, scale = _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, tile=tile)
    assert err <= 0.02 * scale, (tile, case, err, scale)


@pytest.mark.parametrize("tile", list(range(SKN0, N_TILES)))
def test_skinny_dual_stage4(tile):
    """The stage-4 entry's conv3 + downsample (512 @7x7 + 1024 @14x14 / 2 -> 2048) at b1."""
    g = torch.Generator().manual_seed(tile)
    x1 = torch.randn(1, 7, 7, 512, generator=g).to(torch.bfloat16)
    x2 = torch.randn(1, 14, 14, 1024, generator=g).to(torch.bfloat16)
    w = (torch.randn(2048, 1536, generator=g) * 0.03).to(torch.bfloat16)
    b = torch.randn(2048, generator=g)
    ref = ops.conv_dual(x1, x2, w, b, ops.ACT_RELU, 2)
    got = ops.conv_dual(x1.cuda(), x2.cuda(), w.cuda(), b.cuda(), ops.ACT_RELU, 2, tile=tile)
    torch.cuda.synchronize()
    _assert_close(got.cpu(), ref, ("skinny dual", tile))


def _c2f_weights(seed, exact=False):
    g = torch.Generator().manual_seed(seed)
    s1 = ConvSpec.auto(32, 32, 1, 1, 0, ops.ACT_SILU)
    sm = ConvSpec.auto(16, 16, 3, 1, 1, ops.ACT_SILU)
    s2 = ConvSpec.auto(48, 32, 1, 1, 0, ops.ACT_SILU)

    def w(co, ci, k, spec, fan):
        if exact:
            return ops.pack_conv_weight(torch.randint(-1, 2, (co, ci, k, k), generator=g).float() / 8,
                                        spec)
        return ops.pack_conv_weight(torch.randn(co, ci, k, k, generator=g) * (2.0 / fan) ** 0.5, spec)

    def b(n):
        return (torch.randint(-2, 3, (n,), generator=g).float() / 4 if exact
                else torch.randn(n, generator=g) * 0.1)

    return (w(32, 32, 1, s1, 32), b(32), w(16, 16, 3, sm, 144), b(16), w(16, 16, 3, sm, 144),
            b(16), w(32, 48, 1, s2, 48), b(32))


@pytest.mark.parametrize("geom", [
    # (N, H, W, ldx, x_coff, ldy, y_coff)
    (2, 160, 160, 32, 0, 32, 0),     # YOLOv8n b2 as the model runs it
    (3, 80, 80, 48, 8, 64, 16),      # the 80-wide form, channel slices in and out
    (1, 40, 160, 32, 0, 32, 0),      # one strip per image
])
def test_c2f16_fused(geom):
    """v13 fused C2f(32, 32, n=1, shortcut) (ops.c2f16: cv1 -> 3x3 -> 3x3 + shortcut -> cv2
    over the concat, one launch) vs the four reference convs with the same bf16
    intermediates.  The output is NaN-poisoned first: a pixel or channel the kernel skips
    fails, and channels outside the written slice must stay NaN."""
    N, H, W, ldx, xc, ldy, yc = geom
    wts = _c2f_weights(H + N)
    x = _rand((N, H, W, ldx), 7, scale=2.0)
    ref = ops.c2f16(x, *wts, x_coff=xc)
    out = torch.full((N, H, W, ldy), float("nan"), dtype=torch.bfloat16, device="cuda")
    ops.c2f16(x.cuda(), *(t.cuda() for t in wts), out=out, x_coff=xc, y_coff=yc)
    torch.cuda.synchronize()
    got = out.cpu().float()
    inside = got[..., yc:yc + 32]
    assert not torch.isnan(inside).any()
    mask = torch.ones(ldy, dtype=torch.bool)
    mask[yc:yc + 32] = False
    assert torch.isnan(got[..., mask]).all()
    _assert_close(inside, ref, ("c2f16", geom))


def test_c2f16_fused_exact_small_integers():
    """Layout check with exactly representable data: any swapped tap, channel, row-ring slot or
    pixel mapping changes a result by far more than the summation-order noise."""
    N, H, W = 2, 80, 80
    wts = _c2f_weights(11, exact=True)
    g = torch.Generator().manual_seed(3)
    x = torch.randint(-2, 3, (N, H, W, 32), generator=g).to(torch.bfloat16)
    ref = ops.c2f16(x, *wts)
    got = ops.c2f16(x.cuda(), *(t.cuda() for t in wts)).cpu()
    torch.cuda.synchronize()
    d = (got.float() - ref.float()).abs()
    assert d.max().item() <= 2 ** -6 * ref.float().abs().max().item() + 1e-3, d.max()
    assert (d > 0).float().mean().item() < 0.02


def test_c2f16_matches_four_launch_block():
    """The YOLOv8n b2 block: DC2f's fused launch vs its own four-launch path on the GPU."""
    from kvedge_amd.models.yolov8 import DC2f, C2f
    torch.manual_seed(0)
    blk = DC2f(C2f(32, 32, 1, True).eval(), "cuda")
    x = _rand((2, 160, 160, 32), 9).cuda()
    assert blk.fused_ok(x)
    fused = blk(x)
    old = ops.C2F_ENABLED
    ops.C2F_ENABLED = False
    try:
        four = blk(x)
    finally:
        ops.C2F_ENABLED = old
    torch.cuda.synchronize()
    _assert_close(fused.cpu(), four.cpu(), "c2f16 vs four launches")


@pytest.mark.parametrize("tile", [-1] + list(range(6, DIRECT0)) + [NLOOP0, 63, 64] +
                         list(range(XP0, DE0)) + [DE0, SKN0, SKN0 + 8] + list(range(PP0, PP0 + 4)))
@pytest.mark.parametrize("geom", [
    # (N, H, W, skip ld, skip coff, K1, low ld, low coff, K2, Cout, y ld, y coff): YOLO h15 / h12
    (2, 20, 20, 192, 128, 64, 192, 64, 128, 64, 96, 0),
    (1, 10, 12, 384, 256, 128, 384, 128, 256, 128, 192, 64),
])
def test_conv_dual2_up2(tile, geom):
    """The neck's [upsample2x(low) | skip] concat folded into cv1 (ops.conv_dual2, up2): the
    v2 LDS-DMA tiles and their v7 / v8 forms compute it (vs the fp32 reference; channels
    outside the output slice stay untouched), every other family refuses it."""
    N, H, W, lds, sc, K1, ldl, lc, K2, cout, ldy, yc = geom
    g = torch.Generator().manual_seed(tile + 100)
    skip = torch.randn(N, H, W, lds, generator=g).to(torch.bfloat16)
    low = torch.randn(N, H // 2, W // 2, ldl, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, K1 + K2, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(cout, generator=g)
    ref = torch.full((N, H, W, ldy), 7.0, dtype=torch.bfloat16)
    ops.conv_dual2(skip, K1, low, w, b, ops.ACT_SILU, ref, x_coff=sc, x2_coff=lc, y_coff=yc,
                   up2=True)
    out = torch.full((N, H, W, ldy), 7.0, dtype=torch.bfloat16, device="cuda")
    args = (skip.cuda(), K1, low.cuda(), w.cuda(), b.cuda(), ops.ACT_SILU, out)
    kw = dict(x_coff=sc, x2_coff=lc, y_coff=yc, up2=True, tile=tile)
    if not (tile == -1 or 6 <= tile < STREAM0 or XP0 <= tile < DE0 or tile >= PP0):
        with pytest.raises(RuntimeError):
            ops.conv_dual2(*args, **kw)
        return
    ops.conv_dual2(*args, **kw)
    torch.cuda.synchronize()
    got = out.cpu()
    mask = torch.ones(ldy, dtype=torch.bool)
    mask[yc:yc + cout] = False
    assert (got[..., mask].float() == 7.0).all()
    _assert_close(got[..., yc:yc + cout], ref[..., yc:yc + cout], ("dual2 up2", tile, geom))


@pytest.mark.parametrize("tile", list(range(PP0, PP0 + 4)))
@pytest.mark.parametrize("case", [
    # (N, H, W, cin, cout, k, stride, pad, act, res, ldx_extra, x_coff, ldy_extra, y_coff)
    (4, 14, 14, 256, 256, 3, 1, 1, ops.ACT_RELU, False, 0, 0, 0, 0),     # s3 3x3 (36 K-tiles)
    (3, 28, 28, 128, 128, 3, 1, 1, ops.ACT_RELU, False, 0, 0, 0, 0),     # s2 3x3 (the 512 x 128 form)
    (3, 28, 28, 512, 128, 1, 1, 0, ops.ACT_RELU, False, 0, 0, 0, 0),     # s2 reduce
    (2, 7, 7, 512, 512, 3, 1, 1, ops.ACT_RELU, False, 0, 0, 0, 0),       # s4 3x3, M tail
    (3, 14, 14, 512, 512, 3, 2, 1, ops.ACT_RELU, False, 0, 0, 0, 0),     # s4 entry 3x3/2
    (2, 28, 28, 128, 128, 3, 2, 1, ops.ACT_RELU, False, 0, 0, 0, 0),     # K = 1152, 2 tiles of N
    (5, 14, 14, 1024, 256, 1, 1, 0, ops.ACT_RELU, False, 0, 0, 0, 0),    # s3 reduce
    (3, 7, 7, 512, 2048, 1, 1, 0, ops.ACT_RELU, True, 0, 0, 0, 0),       # s4 expand + res
    (2, 9, 11, 192, 136, 1, 1, 0, ops.ACT_NONE, False, 64, 32, 8, 8),    # K / N tails, slices
    (1, 3, 3, 64, 40, 1, 1, 0, ops.ACT_SILU, True, 0, 0, 0, 0),          # one K-tile, tiny M
    # > 256 tiles: the persistent forms walk 2 tiles per workgroup (1x1 K = 256: 4 K-steps,
    # the staging stream crosses a tile boundary every 4; 3x3 K = 2304 with a residual)
    (256, 14, 14, 256, 512, 1, 1, 0, ops.ACT_RELU, True, 0, 0, 0, 0),
    (200, 14, 14, 256, 512, 3, 1, 1, ops.ACT_RELU, False, 0, 0, 0, 0),
])
def test_conv_pp(tile, case):
    """v14 (conv_pp.hip): the 8-phase ping-pong loop at the ResNet-50 GEMM shapes and at K /
    M / N tails, vs the fp32 reference (channels outside the output slice untouched); then
    three launches into NaN-poisoned outputs must agree bitwise: a skipped half-tile, a
    stale LDS read or a restage race shows as NaN or as a launch-to-launch difference."""
    N, H, W, cin, cout, k, s, p, act, res, lx, xc, ly, yc = case
    err, scale = _conv_case(N, H, W, cin, cout, k, s, p, act, res=res, ldx_extra=lx, x_coff=xc,
                            ldy_extra=ly, y_coff=yc, tile=tile)
    assert err <= 0.02 * scale, (tile, case, err, scale)
    # a second launch on the same inputs is bitwise identical (no race in the schedule)
    spec = ConvSpec.auto(cin, cout, k, s, p, act)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, H, W, cin, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(cout, spec.Kpad, generator=g) * 0.05).to(torch.bfloat16).cuda()
    b = torch.randn(cout, generator=g).cuda()
    outs = []
    for _ in range(3):
        o = torch.full((N,) + spec.out_hw(H, W) + (cout,), float("nan"), dtype=torch.bfloat16,
                       device="cuda")
        ops.conv2d(x, spec, w, b, out=o, tile=tile)
        outs.append(o)
    torch.cuda.synchronize()
    assert not torch.isnan(outs[0].float()).any()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
