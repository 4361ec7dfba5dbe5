#!/usr/bin/env python3
"""Full tile x layer timing matrix for ResNet-50's 1x1 (GEMM-mode / dual) convs: every
kernel-family tile that accepts the layer, standalone, with effective HBM bandwidth.
Complements tools/layer_bench.py (which only reports the best tile)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tiles", default="")
    ap.add_argument("--only", default="")
    ap.add_argument("--concurrent", type=int, default=1,
                    help="launch each call on this many streams at once (the multi-stream "
                         "engine's situation) and report time per call")
    ap.add_argument("--graph", action="store_true",
                    help="capture the --iters launches in one hipGraph and time its replay "
                         "(edge batches: a bare launch loop is host-bound near 7 us per call)")
    a = ap.parse_args()
    import torch
    from kvedge_amd import ops
    from kvedge_amd.ops import ConvSpec

    assert ops.load()
    B = a.batch
    # (name, hw, cin, cout, res[, k])
    layers = [("s1.c1a", 56, 64, 64, False), ("s1.c1", 56, 256, 64, False),
              ("s1.c3", 56, 64, 256, True), ("s2.c1a", 56, 256, 128, False),
              ("s2.c1", 28, 512, 128, False), ("s2.c3", 28, 128, 512, True),
              ("s3.c1", 14, 1024, 256, False), ("s3.c3", 14, 256, 1024, True),
              ("s4.c3", 7, 512, 2048, True), ("s4.c1", 7, 2048, 512, False),
              ("s3.c1a", 28, 512, 256, False), ("s4.c1a", 14, 1024, 512, False), ("s1.c3-nores", 56, 64, 256, False),
              ("s2.c3-nores", 28, 128, 512, False), ("s3.c3-nores", 14, 256, 1024, False), ("s1.c1a-wide", 56, 64, 512, False),
              ("s1.c2", 56, 64, 64, False, 3), ("s2.c2", 28, 128, 128, False, 3),
              ("s3.c2", 14, 256, 256, False, 3), ("s4.c2", 7, 512, 512, False, 3),
              # stride-2 3x3 (block 0 of stages 2-4): input hw, output hw / 2
              ("s2.c2s", 56, 128, 128, False, 3, 2), ("s3.c2s", 28, 256, 256, False, 3, 2),
              ("s4.c2s", 14, 512, 512, False, 3, 2)]
    if a.only:
        layers = [l for l in layers if l[0] in a.only.split(",")]
    ntiles = int(torch.ops.kvedge.conv_num_tiles())
    tiles = [int(t) for t in a.tiles.split(",")] if a.tiles else list(range(ntiles))

    side = [torch.cuda.Stream() for _ in range(a.concurrent)]

    def timeit_graph(fn):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(5):
            g.replay()
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / (5 * a.iters) * 1e3

    def timeit(fn):
        if a.graph:
            return timeit_graph(fn)
        for _ in range(3):
            fn()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        cur = torch.cuda.current_stream()
        st.record()
        for _ in range(a.iters):
            if a.concurrent == 1:
                fn()
                continue
            for s_ in side:
                s_.wait_stream(cur)
                with torch.cuda.stream(s_):
                    fn()
            for s_ in side:
                cur.wait_stream(s_)
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / a.iters / a.concurrent * 1e3

    print("| layer | " + " | ".join(str(t) for t in tiles) + " | best |")
    print("|---" * (len(tiles) + 2) + "|")
    for name, hw, cin, cout, res, *kk in layers:
        k = kk[0] if kk else 1
        st = kk[1] if len(kk) > 1 else 1
        spec = ConvSpec.auto(cin, cout, k, st, k // 2, ops.ACT_RELU)
        x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
        w = (torch.randn(cout, spec.Kpad, device="cuda") * 0.05).to(torch.bfloat16)
        b = torch.randn(cout, device="cuda")
        ho = hw // st
        out = torch.empty(B, ho, ho, cout, device="cuda", dtype=torch.bfloat16)
        r = torch.randn(B, ho, ho, cout, device="cuda").to(torch.bfloat16) if res else None
        byts = 2.0 * B * (hw * hw * cin + ho * ho * cout * (2 if res else 1)) + 2.0 * cout * spec.Kpad
        flops = 2.0 * B * ho * ho * cout * cin * k * k
        cells, best = [], 1e30
        for t in tiles:
            try:
                us = timeit(lambda: ops.conv2d(x, spec, w, b, res=r, out=out, tile=t))
            except RuntimeError:
                cells.append("-")
                continue
            best = min(best, us)
            cells.append(f"{us:.1f}")
        print(f"| {name} | " + " | ".join(cells) + f" | {byts / best / 1e3:.0f} GB/s "
              f"{flops / best / 1e6:.0f} TF/s |", flush=True)


if __name__ == "__main__":
    main()
