#!/usr/bin/env python3
"""Same-box probe of the v9 bottleneck seam (csrc/kernels/conv_seam.hip) at ResNet-50 shapes.

For each seam shape (stage 2, 2 -> 3, 3, 3 -> 4) at --batch images: every seam tile that
takes the shape, and the unfused pair it replaces (conv3 + residual, then the next conv1),
each conv at its fastest tile of the whole table (the autotuner's choice).  Timings are
medians of interleaved rounds (HIP events around each launch), in microseconds.

  python tools/seam_probe.py --batch 640 > gpurun_out/seam_probe.md
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--rounds", type=int, default=15)
    a = ap.parse_args()
    import torch

    from kvedge_amd import ops
    from kvedge_amd.ops import ConvSpec

    assert ops.load()
    ntiles = int(torch.ops.kvedge.conv_num_tiles())
    nseam = int(torch.ops.kvedge.conv_seam_num_tiles())
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*shape, scale=1.0):
        return (torch.randn(*shape, generator=g, device="cuda") * scale).to(torch.bfloat16)

    def timeit(fns, rounds):
        for f in fns:
            f()
        torch.cuda.synchronize()
        ev = [[] for _ in fns]
        for _ in range(rounds):
            for i, f in enumerate(fns):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                f()
                e.record()
                ev[i].append((s, e))
        torch.cuda.synchronize()
        return [sorted(x.elapsed_time(y) for x, y in v)[len(v) // 2] * 1e3 for v in ev]

    def best_tile(fn):
        ok = []
        for t in range(ntiles):
            try:
                fn(t)
                ok.append(t)
            except RuntimeError:
                pass
        torch.cuda.synchronize()
        ts = timeit([lambda t=t: fn(t) for t in ok], 3)
        i = min(range(len(ok)), key=lambda i: ts[i])
        # re-time the near ties
        near = [ok[j] for j in range(len(ok)) if ts[j] <= ts[i] * 1.15]
        ts2 = timeit([lambda t=t: fn(t) for t in near], 9)
        j = min(range(len(near)), key=lambda j: ts2[j])
        return near[j], ts2[j]

    B = a.batch
    shapes = [("s2 seam", 28, 128, 128), ("s2->s3 seam", 28, 128, 256),
              ("s3 seam", 14, 256, 256), ("s3->s4 seam", 14, 256, 512)]
    base = ntiles
    print(f"# v9 seam probe, batch {B} (us, median of interleaved rounds)\n")
    print("| shape | unfused conv3+res (tile) | unfused conv1 (tile) | unfused sum | "
          "seam tiles (index: us) | best seam | gain |")
    print("|---|---|---|---|---|---|---|")
    for name, hw, k3, n1 in shapes:
        cout = 4 * k3
        t = rnd(B, hw, hw, k3)
        r = rnd(B, hw, hw, cout)
        w3 = rnd(cout, k3, scale=(2.0 / k3) ** 0.5)
        b3 = torch.randn(cout, generator=g, device="cuda") * 0.1
        w1 = rnd(n1, cout, scale=(2.0 / cout) ** 0.5)
        b1 = torch.randn(n1, generator=g, device="cuda") * 0.1
        y = torch.empty(B, hw, hw, cout, dtype=torch.bfloat16, device="cuda")
        z = torch.empty(B, hw, hw, n1, dtype=torch.bfloat16, device="cuda")
        s3 = ConvSpec.auto(k3, cout, 1, 1, 0, ops.ACT_RELU)
        s1 = ConvSpec.auto(cout, n1, 1, 1, 0, ops.ACT_RELU)
        t3, u3 = best_tile(lambda tl: ops.conv2d(t, s3, w3, b3, res=r, out=y, tile=tl))
        t1, u1 = best_tile(lambda tl: ops.conv2d(y, s1, w1, b1, out=z, tile=tl))
        seams = []
        for st in range(nseam):
            try:
                ops.conv_tail(t, w3, b3, ops.ACT_RELU, w1, b1, res=r, out=y, z=z, tile=base + st)
                seams.append(st)
            except RuntimeError:
                pass
        torch.cuda.synchronize()
        fns = [lambda st=st: ops.conv_tail(t, w3, b3, ops.ACT_RELU, w1, b1, res=r, out=y, z=z,
                                           tile=base + st) for st in seams]
        fns.append(lambda: (ops.conv2d(t, s3, w3, b3, res=r, out=y, tile=t3),
                            ops.conv2d(y, s1, w1, b1, out=z, tile=t1)))
        ts = timeit(fns, a.rounds)
        pair = ts[-1]
        bi = min(range(len(seams)), key=lambda i: ts[i]) if seams else None
        cells = ", ".join(f"{st}: {ts[i]:.1f}" for i, st in enumerate(seams))
        best = f"{seams[bi]} ({ts[bi]:.1f})" if bi is not None else "-"
        gain = f"{pair - ts[bi]:+.1f}" if bi is not None else "-"
        print(f"| {name} | {u3:.1f} ({t3}) | {u1:.1f} ({t1}) | {pair:.1f} | {cells} | {best} | {gain} |",
              flush=True)


if __name__ == "__main__":
    main()
