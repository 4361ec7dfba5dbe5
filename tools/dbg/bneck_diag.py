#!/usr/bin/env python3
"""Debug aid for the v11 fused bottleneck: which outputs are unwritten / wrong."""
import sys
import torch

sys.path.insert(0, ".")
from kvedge_amd import ops  # noqa: E402
from kvedge_amd.ops import ConvSpec  # noqa: E402

assert ops.load()
for (N, C, H, W) in [(2, 128, 28, 28), (1, 256, 14, 14)]:
    C4 = 4 * C
    g = torch.Generator().manual_seed(1)
    x = torch.relu(torch.randn(N, H, W, C4, generator=g)).to(torch.bfloat16)
    s1 = ConvSpec.auto(C4, C, 1, 1, 0, ops.ACT_RELU)
    s2 = ConvSpec.auto(C, C, 3, 1, 1, ops.ACT_RELU)
    s3 = ConvSpec.auto(C, C4, 1, 1, 0, ops.ACT_RELU)
    w1 = ops.pack_conv_weight(torch.randn(C, C4, 1, 1, generator=g) * (2.0 / C4) ** 0.5, s1)
    w2 = ops.pack_conv_weight(torch.randn(C, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5, s2)
    w3 = ops.pack_conv_weight(torch.randn(C4, C, 1, 1, generator=g) * (1.0 / C) ** 0.5, s3)
    b1, b2, b3 = (torch.randn(n, generator=g) * 0.1 for n in (C, C, C4))
    ref = ops.bottleneck_fused(x, w1, b1, w2, b2, w3, b3).float()
    out = torch.full((N, H, W, C4), float("nan"), dtype=torch.bfloat16, device="cuda")
    ops.bottleneck_fused(x.cuda(), w1.cuda(), b1.cuda(), w2.cuda(), b2.cuda(), w3.cuda(), b3.cuda(), out=out)
    torch.cuda.synchronize()
    got = out.cpu().float()
    nan = torch.isnan(got)
    print(f"== N{N} C{C} {H}x{W}: nan frac {nan.float().mean():.4f}")
    if nan.any():
        idx = nan.nonzero()
        for d, name in enumerate("nhwc"):
            u = torch.unique(idx[:, d])
            print(f"  nan {name}: {len(u)} distinct, first {u[:20].tolist()} last {u[-5:].tolist()}")
        # per channel-subtile of 32 and per pixel row
        ch = nan.float().mean(dim=(0, 1, 2)).view(-1, 32).mean(1)
        print("  nan frac per 32-ch subtile:", [round(v, 2) for v in ch.tolist()])
        rows = nan.float().mean(dim=(0, 2, 3))
        print("  nan frac per row:", [round(v, 2) for v in rows.tolist()])
    ok = ~nan
    d = (got - ref).abs()
    d[nan] = 0
    print(f"  max err {d.max():.4f} ref max {ref.abs().max():.3f}; rel rms over written "
          f"{((d[ok]**2).mean().sqrt() / (ref[ok]**2).mean().sqrt()).item():.5f}")
    chd = (d.pow(2).mean(dim=(0, 1, 2)) / ref.pow(2).mean(dim=(0, 1, 2)).clamp_min(1e-9)).sqrt()
    print("  rel rms per 32-ch subtile:", [round(v, 3) for v in chd.view(-1, 32).mean(1).tolist()])
    rw = (d.pow(2).mean(dim=(0, 2, 3)) / ref.pow(2).mean(dim=(0, 2, 3)).clamp_min(1e-9)).sqrt()
    print("  rel rms per row:", [round(v, 3) for v in rw.tolist()])
    cl = (d.pow(2).mean(dim=(0, 1, 3)) / ref.pow(2).mean(dim=(0, 1, 3)).clamp_min(1e-9)).sqrt()
    print("  rel rms per col:", [round(v, 3) for v in cl.tolist()])

# phase dumps: z1 (dbg 1) and z2 (dbg 2) of the output pixels vs the reference intermediates
from kvedge_amd.ops import reference as R  # noqa: E402
for (N, C, H, W) in [(2, 128, 28, 28), (1, 256, 14, 14)]:
    C4 = 4 * C
    g = torch.Generator().manual_seed(1)
    x = torch.relu(torch.randn(N, H, W, C4, generator=g)).to(torch.bfloat16)
    s1 = ConvSpec.auto(C4, C, 1, 1, 0, ops.ACT_RELU)
    s2 = ConvSpec.auto(C, C, 3, 1, 1, ops.ACT_RELU)
    s3 = ConvSpec.auto(C, C4, 1, 1, 0, ops.ACT_RELU)
    w1 = ops.pack_conv_weight(torch.randn(C, C4, 1, 1, generator=g) * (2.0 / C4) ** 0.5, s1)
    w2 = ops.pack_conv_weight(torch.randn(C, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5, s2)
    w3 = ops.pack_conv_weight(torch.randn(C4, C, 1, 1, generator=g) * (1.0 / C) ** 0.5, s3)
    b1, b2, b3 = (torch.randn(n, generator=g) * 0.1 for n in (C, C, C4))
    z1 = torch.empty(N, H, W, C, dtype=torch.bfloat16)
    z2 = torch.empty(N, H, W, C, dtype=torch.bfloat16)
    R.conv2d(x, s1, w1, b1, None, z1, 0, 0, 0)
    R.conv2d(z1, s2, w2, b2, None, z2, 0, 0, 0)
    for dbg, want in ((1, z1), (2, z2)):
        out = torch.full((N, H, W, C4), float("nan"), dtype=torch.bfloat16, device="cuda")
        ops.bottleneck_fused(x.cuda(), w1.cuda(), b1.cuda(), w2.cuda(), b2.cuda(), w3.cuda(),
                             b3.cuda(), out=out, _dbg=dbg)
        torch.cuda.synchronize()
        got = out.cpu().float()[..., :C]
        wf = want.float()
        d = (got - wf).abs()
        d[torch.isnan(d)] = 1e9
        bad = d > 0.02 * wf.abs().max() + 1e-3
        print(f"== dbg {dbg} N{N} C{C}: bad frac {bad.float().mean():.4f}")
        if bad.any():
            print("  bad per row:", [round(v, 2) for v in bad.float().mean(dim=(0, 2, 3)).tolist()])
            print("  bad per col:", [round(v, 2) for v in bad.float().mean(dim=(0, 1, 3)).tolist()])
            print("  bad per 8-ch:", [round(v, 2) for v in bad.float().mean(dim=(0, 1, 2)).view(-1, 8).mean(1).tolist()])
            i = bad.nonzero()[0].tolist()
            print("  first bad", i, "got", got[tuple(i)].item(), "want", wf[tuple(i)].item())
