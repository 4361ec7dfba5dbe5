#!/usr/bin/env python3
"""Per-layer timing of the implicit-GEMM conv kernel on every distinct ResNet-50 conv
(and optionally YOLOv8n), against torch/MIOpen on the same shapes.

For each layer: best-of tiles (and the heuristic's pick), TFLOP/s, effective GB/s
(compulsory bytes: input + weights + output [+ residual]), and MIOpen's time.
Writes a markdown table (stdout and --out)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/layer_bench.md")
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()
    import torch
    import torch.nn.functional as F

    from kvedge_amd import ops
    from kvedge_amd.models.resnet import KvResNet50, init_resnet50

    assert ops.load()
    kv = KvResNet50(init_resnet50(0, calibrate=False), "cuda")
    B = a.batch
    # (name, conv, H_in, has_res)
    layers = []
    h = 224
    layers.append(("stem", kv.stem, h // 2, False))  # s2d stem runs on the 112x112x16 input
    h = 56
    seen = set()
    for i, b in enumerate(kv.blocks):
        for nm, c, hin, res in (("c1", b.c1, h, False), ("c2", b.c2, h, False)):
            layers.append((f"b{i}.{nm}", c, hin, res))
        h2 = b.c2.spec.out_hw(h, h)[0]
        layers.append((f"b{i}.c3", b.c3, h2, True))
        if b.down is not None:
            layers.append((f"b{i}.down", b.down, h, False))
        h = h2
    layers.append(("fc", kv.fc, 1, False))

    def timeit(fn):
        for _ in range(3):
            fn()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        st.record()
        for _ in range(a.iters):
            fn()
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / a.iters * 1e3  # us

    rows = []
    tot_best = tot_heur = tot_torch = 0.0
    ntiles = torch.ops.kvedge.conv_num_tiles()
    for name, c, hin, res in layers:
        s = c.spec
        key = (s.cin, s.cout, s.kh, s.stride, hin, res)
        count = sum(1 for (_, c2, h2, r2) in layers
                    if (c2.spec.cin, c2.spec.cout, c2.spec.kh, c2.spec.stride, h2, r2) == key)
        if key in seen:
            continue
        seen.add(key)
        x = torch.randn(B, hin, hin, s.cin_eff, device="cuda").to(torch.bfloat16)
        Ho, Wo = s.out_hw(hin, hin)
        out = torch.empty(B, Ho, Wo, s.cout, device="cuda", dtype=torch.bfloat16)
        r = torch.randn(B, Ho, Wo, s.cout, device="cuda").to(torch.bfloat16) if res else None
        t_heur = timeit(lambda: ops.conv2d(x, s, c.w, c.b, res=r, out=out))
        best, best_t = None, 1e30
        for t in range(ntiles):
            tt = timeit(lambda: ops.conv2d(x, s, c.w, c.b, res=r, out=out, tile=t))
            if tt < best_t:
                best, best_t = t, tt
        flops = 2.0 * B * Ho * Wo * s.cout * s.kh * s.kw * s.cin
        byts = 2.0 * (B * hin * hin * s.cin_eff + s.cout * s.Kpad + B * Ho * Wo * s.cout *
                      (2 if res else 1))
        t_torch = float("nan")
        if not a.no_torch:
            xt = x[..., :s.cin].permute(0, 3, 1, 2)
            wt = ops.unpack_conv_weight(c.w, s).cuda().to(torch.bfloat16).to(
                memory_format=torch.channels_last)
            xt = xt.contiguous(memory_format=torch.channels_last)
            bt = c.b.to(torch.bfloat16)
            rt = r.permute(0, 3, 1, 2) if r is not None else None

            def tf():
                y = F.conv2d(xt, wt, bt, s.stride, s.pad)
                if rt is not None:
                    y = y + rt
                return F.relu(y)
            t_torch = timeit(tf)
        rows.append((name, count, f"{s.cin}->{s.cout} k{s.kh}s{s.stride} @{hin}", res, t_heur,
                     best, best_t, flops / best_t / 1e6, byts / best_t / 1e3, t_torch))
        tot_best += best_t * count
        tot_heur += t_heur * count
        if t_torch == t_torch:
            tot_torch += t_torch * count
    lines = [f"# ResNet-50 layer bench, batch {B}", "",
             "| layer | x | shape | res | heur us | best tile | best us | TF/s | GB/s | torch us |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for r_ in rows:
        lines.append("| %s | %d | %s | %s | %.1f | %d | %.1f | %.0f | %.0f | %.1f |" % r_)
    lines.append("")
    lines.append(f"total conv time (x count): heuristic {tot_heur:.0f} us, best-tile {tot_best:.0f} us, "
                 f"torch {tot_torch:.0f} us")
    txt = "\n".join(lines)
    print(txt)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        f.write(txt + "\n")


if __name__ == "__main__":
    main()
