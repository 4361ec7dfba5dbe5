"""ResNet-50 v1.5 (torchvision layout) — reference NCHW module and deployed NHWC bf16 form.

North-star flagship model (BASELINE.json config 2/3).  The
reference repository has no model code; this is a new component.  Weights are
random-init with a fixed seed (no checkpoints / no network), optionally with BN
statistics calibrated on synthetic frames so activations stay well scaled.

Deployed forward (all HIP kernels on GPU):
  frames u8 NHWC3 -> ONE stem kernel (normalise + space-to-depth in its fetch, 7x7/2 conv
  as a 4x4 s2d conv with BN+ReLU, 3x3/2 max pool; stem_pool.hip) -> 16 bottlenecks of
  direct / streaming implicit-GEMM convs with bias+residual+ReLU in the epilogue (conv3 and
  the next block's conv1 fused where they fit) -> K6 global avgpool -> K1 FC GEMM ->
  K7 softmax+argmax.
"""
from __future__ import annotations

import os

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .layers import (DeployedConv, DeployedDualConv, calibrate_bn, count_flops, fold_bn,
                     frames_to_nchw)

ACT_NONE, ACT_RELU = ops.ACT_NONE, ops.ACT_RELU
# Stage-1 fused tails (v3 streaming tail tile) only from this many output rows (N*Ho*Wo) up:
# below it (batch <= 10) conv3 and the next conv1 run as separate launches on the edge-batch
# v12 / v1 tiles, which is faster there (same-box A/B, profiles/r5_v8_edge_ab.txt: b1 0.351
# -> 0.336 ms, b8 0.483 -> 0.463 ms with the v12 family's first form).  0 = always fuse.
TAIL1_MIN_ROWS = int(os.environ.get("KVEDGE_TAIL1_MIN_ROWS", "32768"))


# ---------------------------------------------------------------------------
# reference (NCHW fp32)
# ---------------------------------------------------------------------------
class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)  # v1.5: stride on 3x3
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                            nn.BatchNorm2d(cout))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(y + idt)


class ResNet50Ref(nn.Module):
    layers_cfg = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))

    def __init__(self, num_classes: int = 1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        blocks: List[nn.Module] = []
        cin = 64
        for width, n, stride in self.layers_cfg:
            for i in range(n):
                blocks.append(Bottleneck(cin, width, stride if i == 0 else 1))
                cin = width * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(2048, num_classes)
        self.num_classes = num_classes

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.max_pool2d(x, 3, 2, 1)
        x = self.blocks(x)
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)


def init_resnet50(seed: int = 0, num_classes: int = 1000, calibrate: bool = True,
                  calib_batch: int = 4, calib_hw: int = 224) -> ResNet50Ref:
    """Seeded random init (torchvision scheme) + optional BN calibration on synthetic frames."""
    g = torch.Generator().manual_seed(seed)
    m = ResNet50Ref(num_classes)
    for mod in m.modules():
        if isinstance(mod, nn.Conv2d):
            fan_out = mod.out_channels * mod.kernel_size[0] * mod.kernel_size[1]
            with torch.no_grad():
                mod.weight.normal_(0.0, (2.0 / fan_out) ** 0.5, generator=g)
        elif isinstance(mod, nn.BatchNorm2d):
            nn.init.ones_(mod.weight)
            nn.init.zeros_(mod.bias)
        elif isinstance(mod, nn.Linear):
            bound = 1.0 / mod.in_features ** 0.5
            with torch.no_grad():
                mod.weight.uniform_(-bound, bound, generator=g)
                mod.bias.uniform_(-bound, bound, generator=g)
    if calibrate:
        frames = torch.randint(0, 256, (calib_batch, calib_hw, calib_hw, 3), generator=g,
                               dtype=torch.uint8)
        calibrate_bn(m, [frames_to_nchw(frames)])
    m.eval()
    return m


# ---------------------------------------------------------------------------
# deployed (NHWC bf16, HIP kernels)
# ---------------------------------------------------------------------------
class DeployedBottleneck:
    """conv1 -> conv2 -> conv3 with bias+residual+ReLU fused in conv3's epilogue.  Blocks
    with a downsample branch run conv3 and the downsample as ONE GEMM over K = width + cin
    (DeployedDualConv): the downsample output is never materialised (fuse_down=True)."""

    def __init__(self, b: Bottleneck, device, fuse_down: bool = True):
        self.c1 = DeployedConv.from_modules(b.conv1, b.bn1, ACT_RELU, device)
        self.c2 = DeployedConv.from_modules(b.conv2, b.bn2, ACT_RELU, device)
        self.c3 = DeployedConv.from_modules(b.conv3, b.bn3, ACT_RELU, device)
        self.down = None
        self.dual = None
        if b.downsample is not None:
            self.down = DeployedConv.from_modules(b.downsample[0], b.downsample[1], ACT_NONE,
                                                  device)
            if fuse_down:
                self.dual = DeployedDualConv.from_modules(b.conv3, b.bn3, b.downsample[0],
                                                          b.downsample[1], ACT_RELU, device)

    def __call__(self, x, out=None, t1=None):
        """t1: this block's conv1 output when a previous fused tail already computed it."""
        y = self.c1(x) if t1 is None else t1
        y = self.c2(y)
        if self.dual is not None:
            return self.dual(y, x, out=out)
        idt = x if self.down is None else self.down(x)
        return self.c3(y, res=idt, out=out)

    def can_tail(self, nxt: "DeployedBottleneck") -> bool:
        """conv3 (or the fused downsample GEMM) + the next block's conv1 as one fused tail.
        Stage 1 (Cout = 256): the v3 tail tile holds a whole y row and both weight slices in
        LDS.  Stages 2-3 (plain conv3 + residual, K3 = 128 / 256): the v9 seam kernel
        (conv_seam.hip) walks the y tiles with conv3's A resident and keeps the next conv1's
        z in registers (ops.SEAM_SHAPES; KVEDGE_SEAM=0 turns it off for A/Bs)."""
        c1 = nxt.c1.spec
        cout = self.c3.spec.cout
        if not (c1.kh == 1 and c1.stride == 1 and c1.pad == 0 and c1.cin == cout and
                c1.act == ACT_RELU and self.c3.spec.act == ACT_RELU):
            return False
        if cout != 256:
            k3 = self.c3.spec.cin
            return (ops.SEAM_ENABLED and self.down is None and self.dual is None and
                    (k3, cout, c1.cout) in ops.SEAM_SHAPES)
        k = self.c3.spec.cin + (self.dual.w.shape[1] - self.dual.k1 if self.dual is not None else 0)
        return (c1.cout in (64, 128) and (self.dual is not None or self.down is None) and
                (self.dual is None or c1.cout == 64) and k <= 128)

    def tail_fits(self, x: torch.Tensor, batch: int = 0) -> bool:
        """Batch-size gate of the fused boundary for input ``x``: the v9 seam gives each
        8-wave workgroup 128 rows and walks every y tile in it, so it only pays when the
        layer has rows for a workgroup on every CU (ops.SEAM_MIN_WGS); edge batches keep
        the split-K conv3 and conv1 launches.  The stage-1 tail has no such limit.
        ``batch``: gate on this batch instead of x's (micro-batches use the FULL batch, so
        both paths fuse the same boundaries and round y the same way -- ADVICE r4)."""
        N, Ho, Wo, _ = self.out_shape(x.shape)
        N = batch or N
        if self.c3.spec.cout == 256:
            return N * Ho * Wo >= TAIL1_MIN_ROWS
        return (N * Ho * Wo + 127) // 128 >= ops.SEAM_MIN_WGS

    def call_tail(self, x, nxt: "DeployedBottleneck", t1=None, out=None, z=None):
        """-> (this block's output y, the next block's conv1 output z) in one fused pass.
        ``out``/``z``: preallocated destinations (micro-batch slices of full-batch tensors)."""
        y = self.c1(x) if t1 is None else t1
        y = self.c2(y)
        c1 = nxt.c1
        if self.dual is not None:
            d = self.dual
            return ops.conv_tail(y, d.w, d.b, d.act, c1.w, c1.b, x2=x, stride2=d.stride2,
                                 out=out, z=z)
        return ops.conv_tail(y, self.c3.w, self.c3.b, self.c3.spec.act, c1.w, c1.b, res=x,
                             out=out, z=z)

    def out_shape(self, x_shape):
        N, H, W, _ = x_shape
        Ho, Wo = self.c2.spec.out_hw(H, W)
        return (N, Ho, Wo, self.c3.spec.cout)

    def convs(self):
        return [c for c in (self.c1, self.c2, self.c3, self.down, self.dual) if c is not None]


class KvResNet50:
    """Deployed ResNet-50: frames (u8 NHWC3) -> (probs fp32 [B,C], top1 int64 [B])."""

    image_size = 224

    def __init__(self, ref: ResNet50Ref, device="cuda"):
        self.device = torch.device(device)
        self.num_classes = ref.num_classes
        # stride-2 7x7 stem as a stride-1 4x4 conv over space-to-depth input (K12b)
        self.stem = DeployedConv.stem_s2d(ref.conv1, ref.bn1, ACT_RELU, self.device)
        # the same folded stem as a 12-channel s2d 4x4 conv (K = 192): the frames-in GPU path
        wf, _ = fold_bn(ref.conv1, ref.bn1)
        self.stem12_w = ops.pack_stem12(wf).to(self.device)
        self._flops = {}
        self._ref = ref
        self.blocks = [DeployedBottleneck(b, self.device) for b in ref.blocks]
        fcw = ref.fc.weight.detach().float()[:, :, None, None]
        fc_conv = nn.Conv2d(2048, ref.num_classes, 1, bias=True)
        with torch.no_grad():
            fc_conv.weight.copy_(fcw)
            fc_conv.bias.copy_(ref.fc.bias.detach())
        self.fc = DeployedConv.from_modules(fc_conv, None, ACT_NONE, self.device)

    @staticmethod
    def build(seed: int = 0, device="cuda", calibrate: bool = True) -> "KvResNet50":
        return KvResNet50(init_resnet50(seed, calibrate=calibrate), device)

    def convs(self) -> List[DeployedConv]:
        out = [self.stem]
        for b in self.blocks:
            out += b.convs()
        return out + [self.fc]

    def flops_per_image(self, hw: int = 224) -> int:
        """Model FLOPs (2*MAC of all convs + FC) of the reference architecture."""
        if hw not in self._flops:
            self._flops[hw] = count_flops(self._ref, (1, 3, hw, hw))
        return self._flops[hw]

    def preprocess(self, frames_u8: torch.Tensor) -> torch.Tensor:
        return ops.preprocess(frames_u8, s2d=True)

    # Early, memory-bound stages run in micro-batches so their activations stay resident
    # in the 256 MiB Infinity Cache between layers (a 256-image layer1 tensor is 411 MB,
    # a 32-image one 51 MB); the compute-bound late stages run on the whole batch.
    microbatch: int = 0          # 0 = off
    microbatch_blocks: int = 3   # bottlenecks (from the start) run per micro-batch
    fuse_stem_pool: bool = True  # stem conv + max pool as one kernel (stem_pool.hip)
    # GPU: raw frames straight into the stem kernel (preprocess fused into its fetch)
    fuse_preprocess: bool = True
    # conv3 (+ fused downsample) and the NEXT block's conv1 as one kernel wherever the
    # tail tile fits (layer1 -> layer2 boundary included): y is never re-read from HBM
    fuse_tail: bool = True
    # frames-in stem: the 12-channel s2d kernel (stem12.hip, K 192, two workgroups per CU)
    # instead of the 16-channel one (stem_pool.hip, K 256)
    stem12: bool = True

    def stem_and_pool(self, x: torch.Tensor, frames_in: bool = False) -> torch.Tensor:
        if frames_in:
            if self.stem12:
                return ops.stem12_pool_frames(x, self.stem12_w, self.stem.b)
            return ops.stem_pool_frames(x, self.stem.spec, self.stem.w, self.stem.b)
        if self.fuse_stem_pool:
            return ops.stem_pool(x, self.stem.spec, self.stem.w, self.stem.b)
        return ops.maxpool2d(self.stem(x), 3, 2, 1)

    def features(self, x: torch.Tensor, frames_in: bool = False) -> torch.Tensor:
        """x: preprocessed bf16 s2d [B,112,112,16] (or, with ``frames_in``, the raw uint8
        frames [B,224,224,3]) -> final feature map [B,7,7,2048] bf16."""
        B = x.shape[0]
        mb = self.microbatch
        nb = self.microbatch_blocks
        t1 = None
        if mb and B > mb and B % mb == 0 and 0 < nb < len(self.blocks):
            full = full_t1 = None
            for i in range(0, B, mb):
                y = self.stem_and_pool(x[i:i + mb], frames_in)
                z = None
                for j in range(nb):
                    b, nxt = self.blocks[j], self.blocks[j + 1]
                    last = j == nb - 1
                    if last and full is None:
                        shp = b.out_shape(y.shape)
                        full = ops.empty((B,) + shp[1:], dtype=y.dtype, device=y.device)
                    # the same batch gate as the whole-batch path below, evaluated on the
                    # FULL batch B: a micro-batch-sized gate would fuse (or not) differently
                    # from the whole-batch path and change y's bf16 rounding
                    fuse = (self.fuse_tail and y.is_cuda and b.can_tail(nxt) and
                            b.tail_fits(y, batch=B))
                    if last and full_t1 is None and fuse:
                        full_t1 = ops.empty(full.shape[:3] + (nxt.c1.spec.cout,),
                                            dtype=y.dtype, device=y.device)
                    # the last micro-batched block writes straight into the full-batch
                    # tensors (and, fused, the next block's conv1 output too)
                    o = full[i:i + mb] if last else None
                    if fuse:
                        y, z = b.call_tail(y, nxt, t1=z, out=o,
                                           z=full_t1[i:i + mb] if last else None)
                    else:
                        y, z = b(y, t1=z, out=o), None
            x, t1 = full, full_t1
            rest = self.blocks[nb:]
        else:
            x = self.stem_and_pool(x, frames_in)
            rest = self.blocks
        for i, b in enumerate(rest):
            nxt = rest[i + 1] if i + 1 < len(rest) else None
            if (self.fuse_tail and x.is_cuda and nxt is not None and b.can_tail(nxt) and
                    b.tail_fits(x)):
                x, t1 = b.call_tail(x, nxt, t1=t1)
            else:
                x, t1 = b(x, t1=t1), None
        return x

    def logits(self, x: torch.Tensor, frames_in: bool = False) -> torch.Tensor:
        f = self.features(x, frames_in)
        B = f.shape[0]
        if f.is_cuda and B <= ops.POOLED_FC_MAX_BATCH and self.fuse_head:
            return ops.pooled_fc(f, self.fc.w, self.fc.b)  # one GEMV launch at edge batches
        pooled = ops.global_avgpool(f).view(B, 1, 1, 2048)
        return self.fc(pooled).view(B, self.num_classes)

    # edge batches: avgpool + fc as one GEMV kernel (ops.pooled_fc), opt-in with
    # KVEDGE_FUSE_HEAD=1 until it has a same-box edge A/B (the GPU pool gave no box for one)
    fuse_head: bool = os.environ.get("KVEDGE_FUSE_HEAD", "0") == "1"

    def raw_outputs(self, frames_u8: torch.Tensor) -> torch.Tensor:
        """uint8 frames -> pre-softmax logits [B, C] (same kernel path as __call__); the
        cross-replica determinism check (C4) hashes these, not the probabilities."""
        if self.fuse_preprocess and self.fuse_stem_pool and frames_u8.is_cuda:
            return self.logits(frames_u8, frames_in=True)
        return self.logits(self.preprocess(frames_u8))

    def __call__(self, frames_u8: torch.Tensor, out: Optional[dict] = None):
        lg = self.raw_outputs(frames_u8)
        probs, top1 = ops.softmax_rows(lg)
        return probs, top1
