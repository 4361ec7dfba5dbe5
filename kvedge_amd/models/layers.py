"""Model-building blocks shared by ResNet-50 and YOLOv8n.

A model is defined twice, on purpose:
  * a plain ``torch.nn`` NCHW fp32 reference (random-init, seeded) that is the
    numerics oracle and the source of the weights;
  * a *deployed* form: BN folded into conv weight/bias (K4 one-shot fold), weights
    packed [Cout, Kpad] bf16 for the implicit-GEMM kernel, activations NHWC bf16.
The deployed forward calls only :mod:`kvedge_amd.ops` (HIP kernels on GPU).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from ..ops import ConvSpec


def fold_bn(conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d]):
    """Return (weight OIHW fp32, bias fp32) of conv followed by eval-mode BN."""
    w = conv.weight.detach().float()
    b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(w.shape[0])
    if bn is None:
        return w.clone(), b.clone()
    inv = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
    wf = w * inv[:, None, None, None]
    bf = (b - bn.running_mean.detach().float()) * inv + bn.bias.detach().float()
    return wf, bf


_RECORDER: Optional[list] = None


class record_convs:
    """Context manager: record every DeployedConv call (for the tile autotuner)."""

    def __enter__(self):
        global _RECORDER
        _RECORDER = []
        return _RECORDER

    def __exit__(self, *exc):
        global _RECORDER
        _RECORDER = None


def _recorder_active() -> bool:
    return _RECORDER is not None


def _record(layer, key, fn) -> None:
    """Record a fused layer's call for the autotuner (``layer.tile`` is what it pins)."""
    _RECORDER.append((layer, key, fn))


@dataclass
class DeployedConv:
    """A conv ready for the kernel: spec + packed bf16 weight + fp32 bias.

    ``tile`` is the kernel tile index chosen by the autotuner (-1 = heuristic)."""
    spec: ConvSpec
    w: torch.Tensor
    b: torch.Tensor
    tile: int = -1

    @staticmethod
    def from_modules(conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d], act: int,
                     device="cpu") -> "DeployedConv":
        wf, bf = fold_bn(conv, bn)
        cout, cin, kh, kw = wf.shape
        assert kh == kw and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
        spec = ConvSpec.auto(cin, cout, kh, conv.stride[0], conv.padding[0], act)
        return DeployedConv(spec, ops.pack_conv_weight(wf, spec).to(device),
                            bf.contiguous().to(device))

    @staticmethod
    def stem_s2d(conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d], act: int,
                 device="cpu", in_scale: float = 1.0) -> "DeployedConv":
        """Stride-2 KxK stem on RGB -> stride-1 ceil(K/2)... tap conv over the
        space-to-depth input [N, H/2, W/2, 16] written by ops.preprocess(s2d=True).

        out[ho] = sum_r w[r] x[2 ho - p + r].  With X'[by, dy] = x[2 by + dy] and
        q = (p + 1) // 2:  r = 2a + dy + p - 2q, by = ho - q + a, a in [0, ka).
        Taps with r outside [0, K) get zero weight.  Top/left pad q; bottom/right pad
        ka - 1 - q keeps Ho = H/2.  Every 8-element MFMA k-chunk is then one aligned
        16-B load (2 pixels x 4 channels), i.e. the general implicit-GEMM path.

        ``in_scale`` folds an input scale into the weights: 1/255 gives the frames-in
        form (ops.stem_from_frames) that reads raw 0..255 pixel values."""
        wf, bf = fold_bn(conv, bn)
        wf = wf * in_scale
        cout, cin, k, _ = wf.shape
        p, s = conv.padding[0], conv.stride[0]
        assert s == 2 and cin <= 4 and conv.padding[0] == conv.padding[1]
        q = (p + 1) // 2
        ka = (k - 1 + 2 * q - p) // 2 + 1
        w2 = torch.zeros(cout, 16, ka, ka)
        for a in range(ka):
            for dy in range(2):
                r = 2 * a + dy + p - 2 * q
                if not 0 <= r < k:
                    continue
                for b in range(ka):
                    for dx in range(2):
                        t = 2 * b + dx + p - 2 * q
                        if not 0 <= t < k:
                            continue
                        ch = (dy * 2 + dx) * 4
                        w2[:, ch:ch + cin, a, b] = wf[:, :, r, t]
        spec = ConvSpec(16, cout, ka, ka, 1, q, act, ops.MODE_GENERAL, pad_b=ka - 1 - q)
        return DeployedConv(spec, ops.pack_conv_weight(w2, spec).to(device),
                            bf.contiguous().to(device))

    def to(self, device) -> "DeployedConv":
        return DeployedConv(self.spec, self.w.to(device), self.b.to(device), self.tile)

    def __call__(self, x, res=None, out=None, x_coff=0, y_coff=0, r_coff=0, tile=None):
        out = ops.conv2d(x, self.spec, self.w, self.b, res=res, out=out, x_coff=x_coff,
                         y_coff=y_coff, r_coff=r_coff, tile=self.tile if tile is None else tile)
        if _RECORDER is not None:
            s = self.spec
            key = ("conv", s.cin, s.cout, s.kh, s.kw, s.stride, s.pad, s.act, s.mode,
                   tuple(x.shape), x_coff, tuple(out.shape), res is not None)
            fn = lambda t, o=out: ops.conv2d(x, s, self.w, self.b, res=res, out=o,  # noqa: E731
                                             x_coff=x_coff, y_coff=y_coff, r_coff=r_coff, tile=t)
            _RECORDER.append((self, key, fn))
        return out

    @property
    def flops_per_pixel(self) -> int:
        s = self.spec
        return 2 * s.kh * s.kw * s.cin * s.cout


@dataclass
class DeployedDualConv:
    """Bottleneck conv3 (+BN) and its downsample conv (+BN) as ONE GEMM over the
    concatenated reduction dim: out = act(y . W3 + x[::s, ::s] . Wd + b3 + bd).
    Replaces a downsample launch plus the residual write + read of its output."""
    w: torch.Tensor          # [Cout, K1 + K2] bf16
    b: torch.Tensor          # [Cout] fp32
    k1: int
    stride2: int
    act: int
    tile: int = -1

    @staticmethod
    def from_modules(conv3, bn3, down_conv, down_bn, act, device="cpu") -> "DeployedDualConv":
        w3, b3 = fold_bn(conv3, bn3)
        wd, bd = fold_bn(down_conv, down_bn)
        assert w3.shape[2:] == (1, 1) and wd.shape[2:] == (1, 1)
        w = torch.cat([w3[:, :, 0, 0], wd[:, :, 0, 0]], 1)
        return DeployedDualConv(w.to(torch.bfloat16).contiguous().to(device),
                                (b3 + bd).contiguous().to(device), w3.shape[1],
                                down_conv.stride[0], act)

    def __call__(self, y, x, out=None, tile=None):
        out = ops.conv_dual(y, x, self.w, self.b, self.act, self.stride2, out=out,
                            tile=self.tile if tile is None else tile)
        if _RECORDER is not None:
            key = ("dual", tuple(y.shape), tuple(x.shape), tuple(self.w.shape), self.stride2,
                   self.act)
            fn = lambda t, o=out: ops.conv_dual(y, x, self.w, self.b, self.act,  # noqa: E731
                                                self.stride2, out=o, tile=t)
            _RECORDER.append((self, key, fn))
        return out

    def flops_per_pixel(self) -> int:
        return 2 * self.w.shape[0] * self.w.shape[1]


@torch.no_grad()
def calibrate_bn(model: nn.Module, batches, momentum: Optional[float] = None) -> None:
    """Set BN running stats from synthetic batches so a random-init network is
    well conditioned (activations O(1) through all layers), like a trained one.
    Uses cumulative averaging (momentum=None)."""
    bns = [m for m in model.modules() if isinstance(m, nn.BatchNorm2d)]
    saved = [(m.momentum) for m in bns]
    for m in bns:
        m.reset_running_stats()
        m.momentum = momentum
    model.train()
    for x in batches:
        model(x)
    model.eval()
    for m, mo in zip(bns, saved):
        m.momentum = mo


def frames_to_nchw(frames_u8: torch.Tensor, mean=ops.IMAGENET_MEAN,
                   std=ops.IMAGENET_STD) -> torch.Tensor:
    """uint8 NHWC3 frames -> normalized fp32 NCHW (reference path)."""
    x = frames_u8.float() / 255.0
    x = (x - torch.tensor(mean, device=x.device)) / torch.tensor(std, device=x.device)
    return x.permute(0, 3, 1, 2).contiguous()


def count_flops(module: nn.Module, input_shape) -> int:
    """2*MAC FLOPs of every Conv2d/Linear for one forward of ``input_shape`` (NCHW),
    evaluated on the meta device (no compute, no weights touched)."""
    import copy

    m = copy.deepcopy(module).to("meta").eval()
    total = [0]

    def hook(mod, inp, out):
        if isinstance(mod, nn.Conv2d):
            kh, kw = mod.kernel_size
            total[0] += 2 * out.numel() * (mod.in_channels // mod.groups) * kh * kw
        elif isinstance(mod, nn.Linear):
            total[0] += 2 * out.numel() * mod.in_features

    hs = [x.register_forward_hook(hook) for x in m.modules()
          if isinstance(x, (nn.Conv2d, nn.Linear))]
    with torch.no_grad():
        m(torch.empty(*input_shape, device="meta"))
    for h in hs:
        h.remove()
    return total[0] // input_shape[0]
