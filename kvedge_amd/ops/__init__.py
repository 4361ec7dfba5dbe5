"""kvedge_amd.ops — Python face of the gfx950 HIP kernel library.

Contract
--------
* GPU tensors ALWAYS go to the hand-written HIP kernels in ``kvedge_amd/_C.so``.
  If the extension is missing on a GPU box the call raises — there is no silent
  eager fallback on the device path.
* CPU tensors go to :mod:`kvedge_amd.ops.reference`, a plain-PyTorch fp32
  implementation of the *same* semantics (NHWC, packed weights, channel slices).
  That path exists so the model/engine/module plumbing is testable without a GPU
  and doubles as the numerics oracle for the kernel tests.

Layout conventions (shared by kernels and reference):
* activations: NHWC bf16, viewed as ``[N, H, W, ld]``; an op may read/write a
  channel slice ``[coff, coff + C)`` of a wider buffer (concat-free YOLO neck).
* conv weights: packed ``[Cout, Kpad]`` bf16, k-order ``(r, s, c)``; BN folded.
  Stem mode (mode 2): input padded to 4 channels, KW padded to even,
  k-order ``(r, s_padded, c4)`` so that each 8-element MFMA k-chunk is two
  adjacent pixels (16 contiguous bytes).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from . import reference as _ref

# KVEDGE_CHECKS=1 selects the bounds-check build (python -m kvedge_amd._build with the
# same variable set): launchers verify operand extents against their HIP allocations.
# KVEDGE_LIB=<file name in kvedge_amd/> selects another in-tree build of the same sources
# (A/B of one kernel change on one box: tools/ab_build.sh)
_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "_C_checks.so" if os.environ.get("KVEDGE_CHECKS", "0") not in ("", "0")
                         else os.path.basename(os.environ.get("KVEDGE_LIB", "") or "_C.so"))
_loaded = False
_load_error: Optional[str] = None

ACT_NONE, ACT_RELU, ACT_SILU = 0, 1, 2
RES_AFTER_ACT = 4  # flag: y = act(conv) + res  (default: y = act(conv + res))
MODE_GENERAL, MODE_GEMM, MODE_STEM = 0, 1, 2
BK = 64


def load(build_if_missing: bool = False) -> bool:
    """Load the native op library once. Returns True when available."""
    global _loaded, _load_error
    if _loaded:
        return True
    if not os.path.exists(_LIB_PATH) and build_if_missing:
        from .. import _build

        _build.build()
    if not os.path.exists(_LIB_PATH):
        _load_error = f"{_LIB_PATH} not built (run `python -m kvedge_amd._build`)"
        return False
    try:
        torch.ops.load_library(_LIB_PATH)
    except Exception as e:  # pragma: no cover - depends on build state
        _load_error = f"failed to load {_LIB_PATH}: {e}"
        return False
    _check_single_hip_runtime()
    global SPLITK0
    SPLITK0 = int(torch.ops.kvedge.conv_splitk_base())
    if int(torch.ops.kvedge.conv_splitk_num_tiles()) != N_SPLITK_TILES:
        _load_error = "split-K tile count differs from the native library (stale build?)"
        return False
    _loaded = True
    return True


def _check_single_hip_runtime() -> None:
    """Two libamdhip64 copies in one process (torch's + system) would split HIP state."""
    try:
        with open("/proc/self/maps") as f:
            libs = {ln.split()[-1] for ln in f if "libamdhip64" in ln}
    except OSError:
        return
    real = {os.path.realpath(p) for p in libs}
    if len(real) > 1:
        raise RuntimeError(f"kvedge: multiple HIP runtimes loaded: {sorted(real)}")


def native_available() -> bool:
    return load()


def library_path() -> str:
    return _LIB_PATH


# ---------------------------------------------------------------------------
# activation allocation (every op/model output goes through here so the native arena
# planner can see tensor lifetimes: kvedge_amd.runtime.plan_memory)
# ---------------------------------------------------------------------------
_recorder = None


def empty(*shape, dtype=None, device=None) -> torch.Tensor:
    t = torch.empty(*shape, dtype=dtype, device=device)
    if _recorder is not None:
        _recorder(t)
    return t


def set_alloc_recorder(fn) -> None:
    """Install (or clear with None) a callback seeing every activation allocation."""
    global _recorder
    _recorder = fn


def _native():
    if not load():
        raise RuntimeError(
            "kvedge_amd native kernels are required for GPU tensors but unavailable: "
            f"{_load_error}")
    return torch.ops.kvedge


# ---------------------------------------------------------------------------
# conv spec + weight packing
# ---------------------------------------------------------------------------
@dataclass
class ConvSpec:
    cin: int
    cout: int
    kh: int
    kw: int
    stride: int = 1
    pad: int = 0
    act: int = ACT_NONE
    mode: int = MODE_GENERAL
    pad_b: int = -1  # bottom/right padding when asymmetric (s2d stem); -1 = same as pad

    @property
    def pad_end(self) -> int:
        return self.pad if self.pad_b < 0 else self.pad_b

    @property
    def cin_eff(self) -> int:
        return 4 if self.mode == MODE_STEM else self.cin

    @property
    def kwp(self) -> int:
        return (self.kw + 1) // 2 * 2

    @property
    def K(self) -> int:
        if self.mode == MODE_STEM:
            return self.kh * self.kwp * 4
        return self.kh * self.kw * self.cin

    @property
    def Kpad(self) -> int:
        return (self.K + BK - 1) // BK * BK

    def out_hw(self, h: int, w: int):
        p = self.pad + self.pad_end
        return ((h + p - self.kh) // self.stride + 1, (w + p - self.kw) // self.stride + 1)

    @staticmethod
    def auto(cin, cout, k, stride=1, pad=None, act=ACT_NONE) -> "ConvSpec":
        if pad is None:
            pad = k // 2
        if cin < 8:
            mode = MODE_STEM
        elif k == 1 and stride == 1 and pad == 0:
            mode = MODE_GEMM
        else:
            mode = MODE_GENERAL
        return ConvSpec(cin, cout, k, k, stride, pad, act, mode)


def pack_conv_weight(w: torch.Tensor, spec: ConvSpec) -> torch.Tensor:
    """torch OIHW fp32 -> packed [Cout, Kpad] bf16 (k-order (r, s, c))."""
    assert w.shape == (spec.cout, spec.cin, spec.kh, spec.kw), (w.shape, spec)
    w = w.detach().float()
    if spec.mode == MODE_STEM:
        wp = torch.zeros(spec.cout, spec.kh, spec.kwp, 4, dtype=torch.float32, device=w.device)
        wp[:, :, :spec.kw, :spec.cin] = w.permute(0, 2, 3, 1)
        flat = wp.reshape(spec.cout, -1)
    else:
        flat = w.permute(0, 2, 3, 1).reshape(spec.cout, -1)
    out = torch.zeros(spec.cout, spec.Kpad, dtype=torch.float32, device=w.device)
    out[:, :flat.shape[1]] = flat
    return out.to(torch.bfloat16).contiguous()


def unpack_conv_weight(wp: torch.Tensor, spec: ConvSpec) -> torch.Tensor:
    """Inverse of :func:`pack_conv_weight` -> OIHW fp32 (bf16-rounded values)."""
    wf = wp.float()[:, :spec.K]
    if spec.mode == MODE_STEM:
        w4 = wf.reshape(spec.cout, spec.kh, spec.kwp, 4)[:, :, :spec.kw, :spec.cin]
        return w4.permute(0, 3, 1, 2).contiguous()
    return wf.reshape(spec.cout, spec.kh, spec.kw, spec.cin).permute(0, 3, 1, 2).contiguous()


# ---------------------------------------------------------------------------
# ops
# ---------------------------------------------------------------------------
# Split-K workspaces (v8 tiles): fp32 slabs [ksplit][M][Cout], one per K slice of a tile
# (plain stores; the finalize kernel sums them), one workspace per (device, stream), since
# layers on one stream run in order while the multi-stream engine's slices run concurrently.
# Sized on first use (warm-up, before hipGraph capture) for the largest split (32) that fits
# under SPLITK_MAX_ELEMS; a tile whose slabs do not fit is refused by the launcher (the
# autotuner skips it), so big layers only ever take their smaller splits.
_WS: dict = {}
SPLITK_MAX_ELEMS = 32 << 20  # 128 MB of fp32 per stream at most
SPLITK_MAX_SPLIT = 32        # largest split of conv_sk.hip kSkTiles
N_SPLITK_TILES = 19          # conv_sk.hip kSkTiles
N_DE_TILES = 3               # v10 direct-epilogue tiles (conv_direct.hip): after split-K
N_SKINNY_TILES = 9           # v12 edge-batch tiles (conv_skinny.hip kSknTiles): before v14
SPLITK0 = 1 << 30            # first split-K tile index, set by load()


def is_splitk(tile: int) -> bool:
    return SPLITK0 <= tile < SPLITK0 + N_SPLITK_TILES


def splitk_workspace(device: torch.device, elems: int) -> Optional[torch.Tensor]:
    """The stream's split-K workspace for a layer of ``elems`` = M x Cout outputs (None if
    not even two slabs fit under SPLITK_MAX_ELEMS).

    Allocated ONCE per (device, stream) at the full SPLITK_MAX_ELEMS (128 MB of fp32 --
    noise in 288 GB of HBM) and never replaced: a captured hipGraph holds the raw pointer,
    not the tensor, and torch hands out pooled stream handles round-robin, so a later
    engine or the autotuner can reach the same key.  Growing the buffer would free memory
    a live graph still writes its slabs into."""
    if elems > SPLITK_MAX_ELEMS // 2:
        return None
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _WS.get(key)
    if ws is None:
        ws = torch.empty(SPLITK_MAX_ELEMS, dtype=torch.float32, device=device)
        _WS[key] = ws
    return ws


def conv2d(x: torch.Tensor, spec: ConvSpec, w: torch.Tensor, bias: Optional[torch.Tensor],
           res: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           x_coff: int = 0, y_coff: int = 0, r_coff: int = 0, tile: int = -1) -> torch.Tensor:
    """Fused conv + bias (+ residual) (+ act).  x: [N,H,W,ldx] bf16 -> out [N,Ho,Wo,ldy]."""
    N, H, W, ldx = x.shape
    Ho, Wo = spec.out_hw(H, W)
    if out is None:
        out = empty(N, Ho, Wo, spec.cout, dtype=torch.bfloat16, device=x.device)
    assert out.shape[:3] == (N, Ho, Wo), (out.shape, (N, Ho, Wo))
    ldy = out.shape[3]
    ldr = res.shape[-1] if res is not None else 0
    if x.is_cuda:
        ws = splitk_workspace(x.device, N * Ho * Wo * spec.cout) if is_splitk(tile) else None
        _native().conv(x, w, bias, res, out, N, H, W, spec.cin_eff, ldx, x_coff, Ho, Wo,
                       spec.cout, spec.kh, spec.kw, spec.stride, spec.pad, spec.K, ldy, y_coff,
                       ldr, r_coff, spec.act, spec.mode, tile, ws)
    else:
        _ref.conv2d(x, spec, w, bias, res, out, x_coff, y_coff, r_coff)
    return out


def conv_pair(x: torch.Tensor, spec: ConvSpec, w: torch.Tensor, bias: torch.Tensor,
              w2: torch.Tensor, b2: torch.Tensor, out: torch.Tensor, x_coff: int = 0,
              z_coff: int = 0, tile: int = 0) -> torch.Tensor:
    """Fused YOLO Detect-branch pair: out[..., z_coff : z_coff + C2] =
    act(conv3x3/1(x[..., x_coff:]) + bias) . w2^T + b2, the 3x3's output t kept on chip
    (csrc/kernels/conv_direct.hip, C2 forms).  spec: the 3x3 (stride 1, pad 1); w2: bf16
    [C2, Cout] (the 1x1's packed weight without K padding); tile: direct tile 0-3.
    CPU: the two reference convs in sequence, t rounded to bf16 in between."""
    assert spec.kh == 3 and spec.stride == 1 and spec.pad == 1 and spec.mode == MODE_GENERAL
    C2 = w2.shape[0]
    assert w2.shape[1] == spec.cout and out.shape[:3] == x.shape[:3]
    if x.is_cuda:
        _native().conv_pair(x, w, bias, w2, b2, out, spec.cin, x_coff, z_coff, spec.act, tile)
        return out
    t = torch.empty(*x.shape[:3], spec.cout, dtype=torch.bfloat16)
    _ref.conv2d(x, spec, w, bias, None, t, x_coff, 0, 0)
    z = t.float() @ w2.float().t() + b2.float()
    out[..., z_coff:z_coff + C2] = z.to(out.dtype)
    return out


def conv_dual(x1: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor],
              act: int, stride2: int, out: Optional[torch.Tensor] = None,
              tile: int = -1) -> torch.Tensor:
    """Bottleneck conv3 + downsample in ONE GEMM (K = K1 + K2):
    out = act(x1 . W[:, :K1]^T + x2[::s, ::s] . W[:, K1:]^T + bias), all 1x1.
    The downsample's output tensor is never written or re-read."""
    N, Ho, Wo, K1 = x1.shape
    cout = w.shape[0]
    if out is None:
        out = empty(N, Ho, Wo, cout, dtype=torch.bfloat16, device=x1.device)
    if x1.is_cuda:
        ws = splitk_workspace(x1.device, N * Ho * Wo * cout) if is_splitk(tile) else None
        _native().conv_dual(x1, x2, w, bias, out, stride2, act, tile, ws)
    else:
        _ref.conv_dual(x1, x2, w, bias, act, stride2, out)
    return out


def conv_dual2(x: torch.Tensor, K1: int, x2: torch.Tensor, w: torch.Tensor,
               bias: Optional[torch.Tensor], act: int, out: torch.Tensor, x_coff: int = 0,
               x2_coff: int = 0, y_coff: int = 0, stride2: int = 1, up2: bool = False,
               tile: int = -1) -> torch.Tensor:
    """Dual-source 1x1 GEMM over channel slices: out[..., y_coff : y_coff + Cout] =
    act(x[..., x_coff : x_coff + K1] . W[:, :K1]^T + x2'[..., x2_coff : x2_coff + K2] . W[:, K1:]^T
    + bias), x2' = x2 at ``stride2``, or with ``up2`` x2 (half resolution) upsampled 2x
    nearest -- YOLO's neck C2f cv1 reads its [upsampled | skip] concat without the upsample
    launch or the concat's upsampled half (v2 LDS-DMA tiles and their v7 / v8 forms only)."""
    if x.is_cuda:
        N, Ho, Wo, _ = x.shape
        ws = splitk_workspace(x.device, N * Ho * Wo * w.shape[0]) if is_splitk(tile) else None
        _native().conv_dual2(x, x_coff, K1, x2, x2_coff, w, bias, out, y_coff, stride2,
                             1 if up2 else 0, act, tile, ws)
    else:
        _ref.conv_dual2(x, x_coff, K1, x2, x2_coff, w, bias, act, stride2, up2, out, y_coff)
    return out


def conv_tail(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], act: int,
              w1: torch.Tensor, b1: Optional[torch.Tensor], res: Optional[torch.Tensor] = None,
              x2: Optional[torch.Tensor] = None, stride2: int = 1,
              out: Optional[torch.Tensor] = None, z: Optional[torch.Tensor] = None,
              tile: int = -1):
    """Fused bottleneck tail: y = act(x . W^T + bias + res) -- or, with ``x2``, the dual
    conv3 + downsample GEMM of :func:`conv_dual` -- AND z = ReLU(y . w1^T + b1), the next
    block's 1x1 reduce conv, in one pass: y is written once and never re-read from HBM.
    w: packed [Cout, K] (1x1); w1: packed [n_t, Cout].  Returns (y, z)."""
    N, H, W, _ = x.shape
    cout, nt = w.shape[0], w1.shape[0]
    if out is None:
        out = empty(N, H, W, cout, dtype=torch.bfloat16, device=x.device)
    if z is None:
        z = empty(N, H, W, nt, dtype=torch.bfloat16, device=x.device)
    if x.is_cuda:
        _native().conv_tail(x, x2, w, bias, res, out, w1, b1, z, stride2, act, tile)
        return out, z
    if x2 is not None:
        _ref.conv_dual(x, x2, w, bias, act, stride2, out)
    else:
        spec = ConvSpec.auto(x.shape[3], cout, 1, 1, 0, act)
        _ref.conv2d(x, spec, w, bias, res, out, 0, 0, 0)
    spec1 = ConvSpec.auto(cout, nt, 1, 1, 0, ACT_RELU)
    _ref.conv2d(out, spec1, w1, b1, None, z, 0, 0, 0)
    return out, z


# v9 bottleneck seams (csrc/kernels/conv_seam.hip) the tail path takes: (conv3 K3, conv3
# Cout, next conv1 Cout) -- ResNet-50 stage 2, 2 -> 3 and 3.  The 3 -> 4 boundary seam
# (N1 = 512) is level with the two unfused launches at batch 640 and stays unfused
# (profiles/r4_v2_seam_probe_b640.md)
SEAM_SHAPES = {(128, 512, 128), (128, 512, 256), (256, 1024, 256)}
SEAM_ENABLED = os.environ.get("KVEDGE_SEAM", "1") != "0"
# ... only when the layer gives every CU a 128-row workgroup (edge batches: split-K instead)
SEAM_MIN_WGS = int(os.environ.get("KVEDGE_SEAM_MIN_WGS", "256"))


# v13 fused YOLOv8 C2f(32, 32, n=1, shortcut) (csrc/kernels/c2f_fused.hip): the b2 block at
# 160 x 160.  KVEDGE_C2F=0 = the four-launch path (A/B knob)
C2F_ENABLED = os.environ.get("KVEDGE_C2F", "1") != "0"


def c2f16_strip(H: int, W: int) -> int:
    """Output rows per workgroup of the fused C2f kernel (0 = no form for this shape)."""
    for S in (40, 32, 20, 16, 8, 4):
        if H % S == 0 and W in (80, 160):
            return S
    return 0


def c2f16(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, wm1: torch.Tensor,
          bm1: torch.Tensor, wm2: torch.Tensor, bm2: torch.Tensor, w2: torch.Tensor,
          b2: torch.Tensor, out: Optional[torch.Tensor] = None, x_coff: int = 0,
          y_coff: int = 0, S: int = 0) -> torch.Tensor:
    """YOLOv8 C2f(32, 32, n=1, shortcut) as one pass: t = SiLU(W1 . x + b1) (a = t[:16],
    s = t[16:]), u = SiLU(conv3x3(s) + bm1), v = s + SiLU(conv3x3(u) + bm2),
    y = SiLU(W2 . [a, s, v] + b2).  Packed bf16 weights w1 [32, >=32], wm1 / wm2 [16, >=144]
    (tap-major), w2 [32, >=48]; fp32 biases.  GPU: one launch, t / u / v never leave the chip.
    CPU: the four reference convs with bf16 intermediates (what the kernel keeps in LDS and
    registers, and what the four-launch path writes)."""
    N, H, W, _ = x.shape
    if out is None:
        out = empty(N, H, W, 32, dtype=torch.bfloat16, device=x.device)
    if x.is_cuda:
        _native().c2f16_fused(x, x_coff, w1, b1, wm1, bm1, wm2, bm2, w2, b2, out, y_coff,
                              S or c2f16_strip(H, W))
        return out
    s1 = ConvSpec.auto(32, 32, 1, 1, 0, ACT_SILU)
    sm1 = ConvSpec.auto(16, 16, 3, 1, 1, ACT_SILU)
    sm2 = ConvSpec.auto(16, 16, 3, 1, 1, ACT_SILU | RES_AFTER_ACT)
    s2 = ConvSpec.auto(48, 32, 1, 1, 0, ACT_SILU)
    cat = torch.empty(N, H, W, 48, dtype=torch.bfloat16)
    u = torch.empty(N, H, W, 16, dtype=torch.bfloat16)
    _ref.conv2d(x, s1, w1, b1, None, cat, x_coff, 0, 0)
    _ref.conv2d(cat, sm1, wm1, bm1, None, u, 16, 0, 0)
    _ref.conv2d(u, sm2, wm2, bm2, cat, cat, 0, 32, 16)
    _ref.conv2d(cat, s2, w2, b2, None, out, 0, y_coff, 0)
    return out


def stem_pool(x: torch.Tensor, spec: "ConvSpec", w: torch.Tensor, bias: torch.Tensor,
              out: Optional[torch.Tensor] = None, y_coff: int = 0) -> torch.Tensor:
    """Fused ResNet stem + max pool: maxpool3x3/2(relu(conv_s2d(x) + bias)).

    x: the space-to-depth image [N, H, W, 16] (ops.preprocess(s2d=True)); spec/w/bias:
    the s2d stem DeployedConv (4x4, stride 1, pads 2/1, Cout 64, ReLU).  -> [N, H/2, W/2, 64].
    GPU: one kernel (csrc/kernels/stem_pool.hip), the 112x112x64 stem output never
    touches HBM.  CPU: the reference conv followed by the reference pool."""
    assert spec.cin == 16 and spec.cout == 64 and spec.kh == 4 and spec.stride == 1
    assert spec.pad == 2 and spec.pad_end == 1 and spec.act == ACT_RELU and spec.Kpad == 256
    N, H, W, _ = x.shape
    Hp, Wp = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    if out is None:
        out = empty(N, Hp, Wp, 64, dtype=torch.bfloat16, device=x.device)
    if x.is_cuda:
        _native().stem_pool(x, w, bias, out, y_coff)
    else:
        y = conv2d(x, spec, w, bias)
        maxpool2d(y, 3, 2, 1, out=out, y_coff=y_coff)
    return out


def stem_pool_frames(frames: torch.Tensor, spec: "ConvSpec", w: torch.Tensor,
                     bias: torch.Tensor, out: Optional[torch.Tensor] = None, y_coff: int = 0,
                     mean=None, std=None) -> torch.Tensor:
    """Frames-in ResNet stem + pool: preprocess(s2d) fused into :func:`stem_pool`.

    frames: uint8 [N, H, W, 3] (H even, W % 4 == 0) -> [N, H/4, W/4, 64] (224 -> 56).
    GPU: stem_pool.hip's U8 instantiation -- the patch fetch reads the raw bytes (one
    12-B load per two s2d pixels), normalises and space-to-depths them in registers; the
    bf16 s2d image (32 B/px) is never written.  CPU: the reference preprocess + stem_pool."""
    assert frames.dtype == torch.uint8 and frames.dim() == 4 and frames.shape[3] == 3
    mean = IMAGENET_MEAN if mean is None else mean
    std = IMAGENET_STD if std is None else std
    if not frames.is_cuda:
        return stem_pool(preprocess(frames, mean=mean, std=std, s2d=True), spec, w, bias,
                         out=out, y_coff=y_coff)
    assert spec.cin == 16 and spec.cout == 64 and spec.kh == 4 and spec.stride == 1
    assert spec.pad == 2 and spec.pad_end == 1 and spec.act == ACT_RELU and spec.Kpad == 256
    N, H0, W0, _ = frames.shape
    H, W = H0 // 2, W0 // 2
    if out is None:
        out = empty(N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, 64, dtype=torch.bfloat16,
                    device=frames.device)
    _native().stem_pool_frames(frames, w, bias, out, list(mean), list(std), y_coff)
    return out


def pack_stem12(wf: torch.Tensor) -> torch.Tensor:
    """Folded 7x7/2 stem weights [Cout, 3, 7, 7] -> the 12-channel s2d 4x4 form [Cout, 192]
    bf16 that csrc/kernels/stem12.hip reads.  K index = r*48 + s*12 + dy*6 + dx*3 + c for
    s2d tap (r, s) in 4x4 and s2d channel (dy, dx, c); its weight is
    wf[:, c, 2r-1+dy, 2s-1+dx] (zero where that leaves 0..6)."""
    cout, cin, k, _ = wf.shape
    assert cin == 3 and k == 7
    w = torch.zeros(cout, 4, 4, 2, 2, 3)
    for r in range(4):
        for dy in range(2):
            ky = 2 * r - 1 + dy
            if not 0 <= ky < 7:
                continue
            for s_ in range(4):
                for dx in range(2):
                    kx = 2 * s_ - 1 + dx
                    if 0 <= kx < 7:
                        w[:, r, s_, dy, dx, :] = wf[:, :, ky, kx].float()
    return w.reshape(cout, 192).to(torch.bfloat16).contiguous()


def stem12_reference(frames: torch.Tensor, w12: torch.Tensor, bias: torch.Tensor,
                     mean=None, std=None) -> torch.Tensor:
    """CPU reference of :func:`stem12_pool_frames`, step for step: normalise (fp32) -> bf16,
    12-channel space-to-depth, 4x4 stride-1 conv (pads 2 / 1) in fp32, bf16, ReLU, 3x3/2
    max pool (pad 1)."""
    mean = IMAGENET_MEAN if mean is None else mean
    std = IMAGENET_STD if std is None else std
    N, H0, W0, _ = frames.shape
    Hs, Ws = H0 // 2, W0 // 2
    m = torch.tensor(mean, dtype=torch.float32)
    inv = 1.0 / torch.tensor(std, dtype=torch.float32)
    x = (frames.float() * (inv / 255.0) + (-m * inv)).to(torch.bfloat16).float()
    x = x.view(N, Hs, 2, Ws, 2, 3).permute(0, 1, 3, 2, 4, 5).reshape(N, Hs, Ws, 12)
    xp = torch.nn.functional.pad(x, (0, 0, 2, 1, 2, 1))  # X: 2 left 1 right, Y: 2 top 1 bottom
    cols = xp.unfold(1, 4, 1).unfold(2, 4, 1)            # [N, Hs, Ws, 12, 4(r), 4(s)]
    cols = cols.permute(0, 1, 2, 4, 5, 3).reshape(N, Hs, Ws, 192)
    y = cols @ w12.float().t() + bias.float()
    y = y.to(torch.bfloat16).float().relu()
    y = torch.nn.functional.max_pool2d(y.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    return y.to(torch.bfloat16).contiguous()


def stem12_pool_frames(frames: torch.Tensor, w12: torch.Tensor, bias: torch.Tensor,
                       out: Optional[torch.Tensor] = None, y_coff: int = 0,
                       mean=None, std=None) -> torch.Tensor:
    """Frames-in ResNet stem + ReLU + 3x3/2 max pool over a 12-channel space-to-depth image
    (K = 192 instead of the 16-channel form's 256; csrc/kernels/stem12.hip).
    frames: uint8 [N, H, W, 3] (H even, W % 4 == 0); w12: :func:`pack_stem12`.
    -> [N, H/4, W/4, 64] (224 -> 56).  CPU: :func:`stem12_reference`."""
    assert frames.dtype == torch.uint8 and frames.dim() == 4 and frames.shape[3] == 3
    mean = IMAGENET_MEAN if mean is None else mean
    std = IMAGENET_STD if std is None else std
    N, H0, W0, _ = frames.shape
    Hs, Ws = H0 // 2, W0 // 2
    if out is None:
        out = empty(N, (Hs - 1) // 2 + 1, (Ws - 1) // 2 + 1, 64, dtype=torch.bfloat16,
                    device=frames.device)
    if not frames.is_cuda:
        out[..., y_coff:y_coff + 64] = stem12_reference(frames, w12, bias, mean, std)
        return out
    _native().stem12_pool_frames(frames, w12, bias, out, list(mean), list(std), y_coff)
    return out


def yolo_stem2_fits(frames_shape) -> bool:
    """Shapes the fused YOLO b0 + b1 kernel takes (csrc/kernels/yolo_stem2.hip)."""
    _, H, W, _ = frames_shape
    return H % 4 == 0 and W % 32 == 0 and 0 < W <= 640


def yolo_stem2(frames: torch.Tensor, spec0: "ConvSpec", w0: torch.Tensor, b0: torch.Tensor,
               spec1: "ConvSpec", w1: torch.Tensor, b1: torch.Tensor,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """YOLOv8n b0 (frames-in s2d stem, SiLU) + b1 (3x3/2 16 -> 32, SiLU) in ONE pass: b0's
    [N, H/2, W/2, 16] output stays in LDS (csrc/kernels/yolo_stem2.hip).
    frames: uint8 [N, H, W, 3] with :func:`yolo_stem2_fits`; spec0/w0/b0: a
    DeployedConv.stem_s2d(..., in_scale=1/255); spec1/w1/b1: the 3x3/2 16 -> 32 conv.
    -> [N, H/4, W/4, 32].  CPU: the two reference ops in sequence (bf16 in between)."""
    assert spec0.kh == 2 and spec0.cin == 16 and spec0.cout == 16, spec0
    assert (spec1.kh, spec1.stride, spec1.cin, spec1.cout) == (3, 2, 16, 32), spec1
    assert spec0.act == ACT_SILU and spec1.act == ACT_SILU
    N, H, W, _ = frames.shape
    if out is None:
        out = empty(N, H // 4, W // 4, 32, dtype=torch.bfloat16, device=frames.device)
    if not frames.is_cuda:
        x = stem_from_frames(frames, spec0, w0, b0)
        return conv2d(x, spec1, w1, b1, out=out)
    _native().yolo_stem2(frames, w0, b0, w1, b1, out)
    return out


def stem_from_frames(frames: torch.Tensor, spec: "ConvSpec", w: torch.Tensor,
                     bias: Optional[torch.Tensor], out: Optional[torch.Tensor] = None,
                     tile: int = -1) -> torch.Tensor:
    """Preprocess + space-to-depth + 2x2 s2d stem conv in ONE pass (YOLO b0).

    frames: uint8 [N, H, W, 3]; spec/w/bias: a DeployedConv.stem_s2d(..., in_scale=1/255)
    (weights scaled for raw 0..255 inputs, so the 1/255 normalisation costs nothing).
    GPU: the frames-in v4 direct kernel (csrc/kernels/conv_direct.hip) builds the s2d
    patch from raw bytes in LDS -- the [N, H/2, W/2, 16] bf16 image is never written.
    CPU: the reference preprocess (values 0..255) then the reference conv."""
    assert spec.kh == 2 and spec.stride == 1 and spec.cin == 16, spec
    N, H, W, _ = frames.shape
    if out is None:
        out = empty(N, H // 2, W // 2, spec.cout, dtype=torch.bfloat16, device=frames.device)
    if frames.is_cuda:
        _native().conv_frames_s2d(frames, w, bias, out, spec.act, tile)
        return out
    x = preprocess(frames, mean=(0.0, 0.0, 0.0), std=(1.0 / 255,) * 3, s2d=True)
    return conv2d(x, spec, w, bias, out=out)


def maxpool2d(x: torch.Tensor, k: int, stride: int, pad: int, out: Optional[torch.Tensor] = None,
              C: Optional[int] = None, x_coff: int = 0, y_coff: int = 0) -> torch.Tensor:
    N, H, W, ldx = x.shape
    C = C or (ldx - x_coff)
    Ho = (H + 2 * pad - k) // stride + 1
    Wo = (W + 2 * pad - k) // stride + 1
    if out is None:
        out = empty(N, Ho, Wo, C, dtype=x.dtype, device=x.device)
    if x.is_cuda:
        _native().maxpool2d(x, out, N, H, W, C, ldx, x_coff, out.shape[3], y_coff, k, stride, pad,
                            Ho, Wo)
    else:
        _ref.maxpool2d(x[..., x_coff:x_coff + C], out, C, k, stride, pad, y_coff)
    return out


def sppf_pool(buf: torch.Tensor, C: int) -> torch.Tensor:
    """buf [N,H,W,4C] with x in slice 0 -> fills slices 1..3 with mp5/mp9/mp13."""
    N, H, W, ld = buf.shape
    assert ld == 4 * C
    if buf.is_cuda:
        _native().sppf_pool(buf, N, H, W, C)
    else:
        _ref.sppf_pool(buf, C)
    return buf


def global_avgpool(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    N, H, W, C = x.shape
    if out is None:
        out = empty(N, C, dtype=x.dtype, device=x.device)
    if x.is_cuda:
        _native().global_avgpool(x, out, N, H * W, C)
    else:
        out.copy_(x.float().mean(dim=(1, 2)).to(out.dtype))
    return out


POOLED_FC_MAX_BATCH = 16  # edge batches: the head runs as one GEMV launch up to here


def pooled_fc(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor],
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Classifier head at edge batches in ONE launch: out [N, ncls] bf16 =
    fc(global_avgpool(x)) with the pooled vector rounded to bf16 as global_avgpool stores it.
    x: [N, H, W, C] bf16; w: the fc's packed [ncls, Kpad] bf16 weight (Kpad >= C).
    CPU: global_avgpool then the 1x1 conv reference."""
    N, H, W, C = x.shape
    ncls = w.shape[0]
    if out is None:
        out = empty(N, ncls, dtype=torch.bfloat16, device=x.device)
    if x.is_cuda:
        _native().pooled_fc(x, w, bias, out)
        return out
    pooled = global_avgpool(x).view(N, 1, 1, C)
    spec = ConvSpec(C, ncls, 1, 1, 1, 0, ACT_NONE, MODE_GEMM)
    _ref.conv2d(pooled, spec, w, bias, None, out.view(N, 1, 1, ncls))
    return out


def softmax_rows(x: torch.Tensor, out: Optional[torch.Tensor] = None,
                 argmax: Optional[torch.Tensor] = None):
    if out is None:
        out = empty(x.shape, dtype=torch.float32, device=x.device)
    if argmax is None:
        argmax = empty(x.shape[0], dtype=torch.int64, device=x.device)
    if x.is_cuda:
        _native().softmax_rows(x, out, argmax)
    else:
        xf = x.float()
        out.copy_(torch.softmax(xf, dim=1))
        argmax.copy_(xf.argmax(dim=1))
    return out, argmax


def upsample2x(x: torch.Tensor, out: torch.Tensor, C: Optional[int] = None, x_coff: int = 0,
               y_coff: int = 0):
    N, H, W, ldx = x.shape
    C = C or (ldx - x_coff)
    if x.is_cuda:
        _native().upsample2x(x, out, N, H, W, C, ldx, x_coff, out.shape[3], y_coff)
    else:
        up = x[..., x_coff:x_coff + C].repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)
        out[..., y_coff:y_coff + C] = up
    return out


def yolo_decode(feats: Sequence[torch.Tensor], strides: Sequence[int], nc: int,
                boxes=None, scores=None, cls=None):
    f0, f1, f2 = feats
    N = f0.shape[0]
    hw = [(f.shape[1], f.shape[2]) for f in feats]
    A = sum(h * w for h, w in hw)
    dev = f0.device
    if boxes is None:
        boxes = empty(N, A, 4, dtype=torch.float32, device=dev)
        scores = empty(N, A, dtype=torch.float32, device=dev)
        cls = empty(N, A, dtype=torch.int32, device=dev)
    if f0.is_cuda:
        _native().yolo_decode(f0, f1, f2, hw[0][0], hw[0][1], hw[1][0], hw[1][1], hw[2][0],
                              hw[2][1], strides[0], strides[1], strides[2], nc, boxes, scores, cls)
    else:
        _ref.yolo_decode(feats, strides, nc, boxes, scores, cls)
    return boxes, scores, cls


def nms(boxes, scores, cls, conf: float = 0.25, iou: float = 0.7, max_det: int = 300,
        out=None, count=None):
    N = scores.shape[0]
    if out is None:
        out = empty(N, max_det, 6, dtype=torch.float32, device=scores.device)
        count = empty(N, dtype=torch.int32, device=scores.device)
    if scores.is_cuda:
        _native().nms(boxes, scores, cls, conf, iou, max_det, out, count)
    else:
        _ref.nms(boxes, scores, cls, conf, iou, max_det, out, count)
    return out, count


def synth_frames(out: torch.Tensor, seed: int, step) -> torch.Tensor:
    """On-device synthetic uint8 NHWC3 frames.  ``step`` int or a device int64[1] counter."""
    if out.is_cuda:
        if isinstance(step, torch.Tensor):
            _native().synth_frames_dev(out, step, seed)
        else:
            _native().synth_frames(out, seed, int(step))
    else:
        _ref.synth_frames(out, seed, step)
    return out


IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def preprocess(x: torch.Tensor, out: Optional[torch.Tensor] = None, mean=IMAGENET_MEAN,
               std=IMAGENET_STD, s2d: bool = False) -> torch.Tensor:
    """uint8 NHWC3 frames -> normalized bf16, either NHWC4 (channel 3 zero) or, with
    ``s2d``, space-to-depth [N, H/2, W/2, 16] (channel (dy*2+dx)*4 + c)."""
    N, H, W, _ = x.shape
    if out is None:
        shape = (N, H // 2, W // 2, 16) if s2d else (N, H, W, 4)
        out = empty(shape, dtype=torch.bfloat16, device=x.device)
    if x.is_cuda:
        _native().preprocess(x, out, list(mean), list(std))
    else:
        _ref.preprocess(x, out, mean, std)
    return out


def batchnorm_nhwc(x, scale, shift, relu=False, out=None):
    if out is None:
        out = torch.empty_like(x)
    if x.is_cuda:
        _native().batchnorm_nhwc(x, out, scale, shift, relu)
    else:
        y = x.float() * scale + shift
        out.copy_((y.clamp_min(0) if relu else y).to(out.dtype))
    return out
