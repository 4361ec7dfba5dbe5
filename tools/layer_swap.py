#!/usr/bin/env python3
"""In-graph tile A/B for chosen layers of the bench graph (the manual form of
engine.autotune.graph_refine, with explicit candidate tiles).

Builds the bench engine (same batch / streams / autotune as bench.py), lists every tuned
layer (ordinal, shape key, pick, runner-ups, isolated us), then for each --layers ordinal
and each --tiles candidate re-captures the step with that one tile changed and times it
against the tuned graph, replays interleaved (engine.autotune._ab).  --apply "i=t,j=t"
measures one combined change against the tuned graph.

  python tools/layer_swap.py --model resnet50 --list
  python tools/layer_swap.py --model resnet50 --layers 7 --tiles 29,75,80,82
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--streams", type=int, default=0)
    ap.add_argument("--layers", default="")
    ap.add_argument("--match", default="", help="also every layer whose shape key contains this")
    ap.add_argument("--tiles", default="")
    ap.add_argument("--apply", default="")
    ap.add_argument("--rounds", type=int, default=2, help="A/B repeats per candidate")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args()
    os.environ.setdefault("KVEDGE_GRAPH_REFINE_S", "0")
    import torch
    from kvedge_amd import ops
    from kvedge_amd.engine import BENCH_BATCH, BENCH_STREAMS, InferenceEngine
    from kvedge_amd.engine.autotune import _ab
    from kvedge_amd.models.layers import record_convs

    assert ops.load(), "kvedge native library not loaded"
    if a.model == "resnet50":
        from kvedge_amd.models.resnet import KvResNet50 as M
    else:
        from kvedge_amd.models.yolov8 import KvYoloV8n as M
    model = M.build(seed=0, device="cuda", calibrate=True)
    batch = a.batch or BENCH_BATCH[a.model]
    streams = a.streams or BENCH_STREAMS[a.model]
    eng = InferenceEngine(model, batch, M.image_size, device=torch.device("cuda"), seed=0,
                          streams=streams)
    eng.prepare(warmup=2, autotune=True)
    with record_convs() as rec:
        eng.model(eng.frames[:eng.batch // eng.n_streams])
    torch.cuda.synchronize()
    layers, seen = [], set()
    for layer, key, fn in rec:
        if id(layer) not in seen:
            seen.add(id(layer))
            layers.append((layer, key))
    for i, (l, k) in enumerate(layers):
        print(json.dumps({"ordinal": i, "key": repr(k), "tile": l.tile,
                          "alts": list(getattr(l, "tile_alts", [])),
                          "us": getattr(l, "tile_us", None)}), flush=True)
    if a.list:
        return 0
    base = eng.graph
    rounds = max(4, min(40, int(200.0 / 14.0)))

    def trial(changes, tag):
        old = [(layers[i][0], layers[i][0].tile) for i, _ in changes]
        for i, t in changes:
            layers[i][0].tile = t
        try:
            g, _ = eng.capture()
        except RuntimeError as e:
            for l, t in old:
                l.tile = t
            print(json.dumps({"trial": tag, "error": str(e)[:120]}), flush=True)
            return
        res = []
        for _ in range(a.rounds):
            x, y = _ab(base, g, rounds)
            res.append((x, y))
        for l, t in old:
            l.tile = t
        gains = [round(100.0 * (x - y) / x, 2) for x, y in res]
        print(json.dumps({"trial": tag, "base_ms": [round(x, 4) for x, _ in res],
                          "new_ms": [round(y, 4) for _, y in res], "gain_pct": gains}),
              flush=True)
        del g

    sel = [int(x) for x in a.layers.split(",") if x.strip()]
    if a.match:
        sel += [i for i, (_, k) in enumerate(layers) if a.match in repr(k) and i not in sel]
    for i in sel:
        for t in [int(x) for x in a.tiles.split(",") if x.strip()]:
            if t != layers[i][0].tile:
                trial([(i, t)], f"layer {i} tile {layers[i][0].tile}->{t}")
    if a.apply:
        ch = [tuple(int(v) for v in kv.split("=")) for kv in a.apply.split(",") if kv]
        trial(ch, f"apply {a.apply}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
