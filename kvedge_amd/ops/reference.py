"""Plain-PyTorch fp32 reference of every kvedge kernel (CPU path + numerics oracle).

Semantics mirror csrc/kernels/*.hip exactly (layouts, channel slices, padding,
tie-breaking) so GPU kernel tests can compare against these on the same inputs.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

ACT_NONE, ACT_RELU, ACT_SILU = 0, 1, 2


def _act(y: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return y.clamp_min(0)
    if act == ACT_SILU:
        return y * torch.sigmoid(y)
    return y


def conv2d(x, spec, w, bias, res, out, x_coff=0, y_coff=0, r_coff=0):
    from . import unpack_conv_weight, MODE_STEM

    xin = x[..., x_coff:x_coff + spec.cin_eff].float()
    if spec.mode == MODE_STEM:
        xin = xin[..., :spec.cin]
    wt = unpack_conv_weight(w, spec).to(xin.device)
    xp = F.pad(xin.permute(0, 3, 1, 2), (spec.pad, spec.pad_end, spec.pad, spec.pad_end))
    y = F.conv2d(xp, wt, None, spec.stride, 0).permute(0, 2, 3, 1)
    if bias is not None:
        y = y + bias.float()
    act, post = spec.act & 3, bool(spec.act & 4)
    if res is not None and not post:
        y = y + res[..., r_coff:r_coff + spec.cout].float()
    y = _act(y, act)
    if res is not None and post:
        y = y.to(out.dtype).float() + res[..., r_coff:r_coff + spec.cout].float()
    out[..., y_coff:y_coff + spec.cout] = y.to(out.dtype)
    return out


def maxpool2d(x, out, C, k, stride, pad, y_coff=0):
    xin = x[..., :C].float().permute(0, 3, 1, 2)
    y = F.max_pool2d(xin, k, stride, pad).permute(0, 2, 3, 1)
    out[..., y_coff:y_coff + C] = y.to(out.dtype)
    return out


def sppf_pool(buf, C):
    x = buf[..., :C].float().permute(0, 3, 1, 2)
    y1 = F.max_pool2d(x, 5, 1, 2)
    y2 = F.max_pool2d(y1, 5, 1, 2)
    y3 = F.max_pool2d(y2, 5, 1, 2)
    for i, y in enumerate((y1, y2, y3), start=1):
        buf[..., i * C:(i + 1) * C] = y.permute(0, 2, 3, 1).to(buf.dtype)
    return buf


def yolo_decode(feats, strides, nc, boxes, scores, cls):
    outs_b, outs_s, outs_c = [], [], []
    for f, s in zip(feats, strides):
        N, h, w, ch = f.shape
        ff = f.float().reshape(N, h * w, ch)
        box = ff[..., :64].reshape(N, h * w, 4, 16).softmax(-1)
        dist = (box * torch.arange(16, dtype=torch.float32, device=f.device)).sum(-1)
        ys, xs = torch.meshgrid(torch.arange(h, device=f.device), torch.arange(w, device=f.device),
                                indexing="ij")
        ax = xs.reshape(-1).float() + 0.5
        ay = ys.reshape(-1).float() + 0.5
        b = torch.stack([ax - dist[..., 0], ay - dist[..., 1], ax + dist[..., 2],
                         ay + dist[..., 3]], -1) * s
        logits = ff[..., 64:64 + nc]
        mx, arg = logits.max(-1)
        outs_b.append(b)
        outs_s.append(torch.sigmoid(mx))
        outs_c.append(arg.int())
    boxes.copy_(torch.cat(outs_b, 1))
    scores.copy_(torch.cat(outs_s, 1))
    cls.copy_(torch.cat(outs_c, 1))
    return boxes, scores, cls


def _iou(a, b):
    iw = (torch.minimum(a[..., 2], b[..., 2]) - torch.maximum(a[..., 0], b[..., 0])).clamp_min(0)
    ih = (torch.minimum(a[..., 3], b[..., 3]) - torch.maximum(a[..., 1], b[..., 1])).clamp_min(0)
    inter = iw * ih
    aa = (a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1])
    ab = (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
    return inter / (aa + ab - inter).clamp_min(1e-9)


def nms(boxes, scores, cls, conf, iou, max_det, out, count, max_wh=7680.0):
    """Greedy class-aware NMS; order = score desc, index asc (same as the kernel)."""
    out.zero_()
    N, A = scores.shape
    for n in range(N):
        s = scores[n].float()
        idx = torch.nonzero(s > conf).flatten()
        if idx.numel() == 0:
            count[n] = 0
            continue
        order = sorted(idx.tolist(), key=lambda i: (-float(s[i]), i))
        order = torch.tensor(order, dtype=torch.long)
        b = boxes[n, order].float()
        c = cls[n, order].float()
        bo = b + (c * max_wh)[:, None]
        keep = []
        for i in range(order.numel()):
            if len(keep) >= max_det:
                break
            if keep:
                ious = _iou(bo[i][None], bo[torch.tensor(keep)])
                if bool((ious > iou).any()):
                    continue
            keep.append(i)
        for r, i in enumerate(keep):
            out[n, r, :4] = b[i]
            out[n, r, 4] = s[order[i]]
            out[n, r, 5] = c[i]
        count[n] = len(keep)
    return out, count


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_frames(out, seed, step):
    if isinstance(step, torch.Tensor):  # int64[1] counter, or [2]: counter + done-count slot
        st = int(step[0].item())
        step[0] += 1
    else:
        st = int(step)
    n8 = out.numel() // 8
    i = np.arange(n8, dtype=np.uint64)
    with np.errstate(over="ignore"):
        mix = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (np.uint64(st) * np.uint64(0xD1B54A32D192ED03))
    h = _splitmix64(mix ^ i)
    out.copy_(torch.from_numpy(h.view(np.uint8).copy()).reshape(out.shape))
    return out


def preprocess(x, out, mean, std):
    xf = x.float() / 255.0
    m = torch.tensor(mean, dtype=torch.float32)
    s = torch.tensor(std, dtype=torch.float32)
    y = (xf - m) * (1.0 / s)
    y4 = torch.zeros(*y.shape[:3], 4, dtype=torch.float32)
    y4[..., :3] = y
    if out.shape[-1] == 16:  # space-to-depth: channel (dy*2+dx)*4 + c
        N, H, W, _ = y4.shape
        y4 = y4.view(N, H // 2, 2, W // 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(
            N, H // 2, W // 2, 16)
    out.copy_(y4.to(out.dtype))
    return out


def conv_dual2(x, x_coff, K1, x2, x2_coff, w, bias, act, stride2, up2, out, y_coff):
    K2 = w.shape[1] - K1
    a = x[..., x_coff:x_coff + K1].float()
    b = x2[..., x2_coff:x2_coff + K2].float()
    b = b.repeat_interleave(2, 1).repeat_interleave(2, 2) if up2 else b[:, ::stride2, ::stride2]
    wf = w.float()
    y = a @ wf[:, :K1].t() + b @ wf[:, K1:].t()
    if bias is not None:
        y = y + bias.float()
    out[..., y_coff:y_coff + w.shape[0]] = _act(y, act & 3).to(out.dtype)
    return out


def conv_dual(x1, x2, w, bias, act, stride2, out):
    K1 = x1.shape[-1]
    wf = w.float()
    y = x1.float() @ wf[:, :K1].t() + x2[:, ::stride2, ::stride2].float() @ wf[:, K1:].t()
    if bias is not None:
        y = y + bias.float()
    out.copy_(_act(y, act & 3).to(out.dtype))
    return out
