"""Per-layer tile autotuner for the implicit-GEMM conv kernels.

One instrumented eager forward records every conv call (DeployedConv / DeployedDualConv)
as (layer, shape key, re-run closure) on its live tensors; each distinct key is then
timed with every tile of the kernel tile table -- v1 register-staged and v2 LDS-DMA
families -- (HIP events, median of a few launches) and the fastest valid tile is pinned
on the layer before hipGraph capture.  Tiles a layer cannot use (e.g. the fused
downsample GEMM on a v1 tile) are skipped.  Correctness never depends on the tile
(tests/test_kernels_gpu.py::test_conv_every_tile).
"""
from __future__ import annotations

import json
import os
from typing import Callable, Dict

import torch

from ..models.layers import record_convs


def _hold_gpu(launches: int) -> None:
    """Queue a spin kernel long enough to cover the host's enqueue of ``launches`` layer
    launches, so the timed events bracket GPU execution, not host launch latency.  Without
    it a small (edge-batch) layer measured the Python + HIP launch path -- about 5-10 us per
    kernel -- which, for a split-K tile (GEMM + finalize: two launches), was larger than
    the kernels themselves, and the tuner never picked the split forms at batch 1."""
    torch.cuda._sleep(int(min(5e7, 60_000 * max(1, launches))))  # ~25 us per launch


def _time(fn: Callable[[int], object], tile: int, iters: int) -> float:
    fn(tile)
    _hold_gpu(iters)
    evs = []
    for _ in range(iters):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        fn(tile)
        en.record()
        evs.append((st, en))
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) for s, e in evs)
    return ts[len(ts) // 2]


def _time_concurrent(fn: Callable[[int], object], tile: int, iters: int, streams) -> float:
    """Median ms of ``len(streams)`` launches of ``fn(tile)`` issued together, one per
    stream: the layer as the multi-stream engine runs it, its copies co-resident on the
    CUs (a tile that fills every CU alone can lose to a leaner one under concurrency)."""
    cur = torch.cuda.current_stream()
    fn(tile)
    _hold_gpu(iters * len(streams))
    evs = []
    for _ in range(iters):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for s in streams:
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                fn(tile)
        for s in streams:
            cur.wait_stream(s)
        en.record()
        evs.append((st, en))
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) for s, e in evs)
    return ts[len(ts) // 2]


def _time_interleaved(cands, rounds: int):
    """Median ms per (fn, tile) with the candidates timed round-robin (A B C A B C ...):
    a clock or thermal drift during the measurement then biases every candidate alike,
    where timing each candidate's launches back to back let a drift decide near-ties."""
    for fn, t in cands:
        fn(t)  # warm: code object loaded, first-launch costs out of the way
    _hold_gpu(rounds * len(cands))
    evs = [[] for _ in cands]
    for _ in range(rounds):
        for i, (fn, t) in enumerate(cands):
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            fn(t)
            en.record()
            evs[i].append((st, en))
    torch.cuda.synchronize()
    out = []
    for e in evs:
        ts = sorted(a.elapsed_time(b) for a, b in e)
        out.append(ts[len(ts) // 2])
    return out


def _fleet_mean(rows):
    """Mean over data-parallel ranks of a [keys][tiles] timing matrix (identity when not
    distributed).  +inf (tile invalid for the layer) is the same on every rank."""
    from .. import parallel

    if not rows or not parallel.is_dist():
        return rows
    flat = [x for r in rows for x in r]
    fin = [x if x != float("inf") else 0.0 for x in flat]
    tot = parallel.allreduce_scalars(fin, op="sum")
    world = parallel.info().world_size
    out, i = [], 0
    for r in rows:
        out.append([tot[i + j] / world if r[j] != float("inf") else float("inf")
                    for j in range(len(r))])
        i += len(r)
    return out


def _near_ties(rows, tol: float):
    """[(row, tile)] of every tile within ``tol`` of its row's best, for rows with more
    than one such tile (the re-timing list of the refine phase; deterministic order)."""
    out = []
    for i, ts in enumerate(rows):
        best = min(ts) if ts else float("inf")
        if best == float("inf"):
            continue
        near = [t for t in range(len(ts)) if ts[t] <= best * (1.0 + tol)]
        if len(near) > 1:
            out += [(i, t) for t in near]
    return out


def autotune(model: Callable, example_input: torch.Tensor, iters: int = 5,
             cache_path: str = None, verbose: bool = False, refine_iters: int = None,
             refine_tol: float = 0.15, concurrency: int = 1) -> Dict:
    """Tune every conv of ``model`` for ``example_input``'s shape. Returns {key: (tile, us)}.

    concurrency > 1: time each tile as that many copies launched together on separate
    streams (the multi-stream engine's situation); the near-tie refine pass then does
    the same."""
    if not example_input.is_cuda:
        return {}
    if refine_iters is None:
        refine_iters = int(os.environ.get("KVEDGE_AUTOTUNE_REFINE_ITERS", "20"))
    ntiles = int(torch.ops.kvedge.conv_num_tiles())
    # A/B knob: tune over the first KVEDGE_TILE_LIMIT tiles only (e.g. without a new family).
    # Applied BEFORE the cache signature: a limited run's picks never pass for a full run's
    lim = int(os.environ.get("KVEDGE_TILE_LIMIT", "0"))
    if 0 < lim < ntiles:
        ntiles = lim
    from .. import parallel

    world = parallel.info().world_size if parallel.is_dist() else 1
    sig = _cache_signature(ntiles, concurrency, world)
    cache, cache_alts = {}, {}
    if cache_path and os.path.exists(cache_path):
        try:
            with open(cache_path) as f:
                doc = json.load(f)
            # picks are valid only for the same kernel library, tile table, device,
            # concurrency and world size; anything else (an older build, the old flat
            # format) is ignored
            if isinstance(doc, dict) and doc.get("signature") == sig:
                for k, v in doc.get("picks", {}).items():
                    cache[k] = (v[0], v[1])
                    if len(v) > 2 and isinstance(v[2], list):
                        cache_alts[k] = [int(t) for t in v[2]]
        except (OSError, ValueError, TypeError, IndexError):
            cache, cache_alts = {}, {}
    with record_convs() as rec:
        model(example_input)
    torch.cuda.synchronize()
    # all-or-nothing: the cache is used only if it covers every layer of this model on
    # EVERY rank -- data-parallel ranks must time the same keys (one all-reduce below)
    if cache and not all(repr(key) in cache for _, key, _ in rec):
        cache = {}
    cache = _fleet_cache(cache, [repr(key) for _, key, _ in rec])
    if not cache:
        cache_alts = {}
    results: Dict = {}
    side = [torch.cuda.Stream() for _ in range(concurrency)] if concurrency > 1 else None
    timer = (lambda f, t, n: _time_concurrent(f, t, n, side)) if side else _time
    # phase 1: time every (distinct key, tile) on this GPU; invalid tiles stay +inf
    todo = {}  # key string -> (key, fn, [us per tile])
    for layer, key, fn in rec:
        ks = repr(key)
        if ks in cache or ks in todo:
            continue
        ts = [float("inf")] * ntiles
        for t in range(ntiles):
            try:
                ts[t] = timer(fn, t, iters) * 1e3
            except RuntimeError:  # tile not valid for this layer kind
                continue
        todo[ks] = (key, fn, ts)
    # phase 2 (data-parallel replicas): every rank times the same keys in the same order
    # (same model, same batch), so ONE all-reduce of the timing matrix gives each rank the
    # fleet-mean time per tile and every replica pins the same, less noisy choice -- the
    # job's images/sec is set by the slowest rank, so per-rank tuning noise costs throughput
    fleet = _fleet_mean([v[2] for v in todo.values()])
    # phase 3: near-ties (within ``refine_tol`` of the best, by the fleet mean -- so every
    # rank re-times the same (key, tile) list in the same order) are re-timed with
    # ``refine_iters`` launches each, the candidates of one layer interleaved round-robin; a
    # 5-launch median alone flipped picks between runs (a stage-2 expand layer took a tile
    # 15 % slower in the graph than the runner-up on one box)
    if refine_iters > iters:
        fns = [(ks, fn) for ks, (_, fn, _) in todo.items()]
        cand = [(fns[i][0], fns[i][1], t) for i, t in _near_ties(fleet, refine_tol)]
        if cand:
            times = []
            for ks in dict.fromkeys(c[0] for c in cand):  # per layer, in first-seen order
                grp = [(fn, t) for k, fn, t in cand if k == ks]
                if side:
                    times += [timer(f, t, refine_iters) * 1e3 for f, t in grp]
                else:
                    times += [x * 1e3 for x in _time_interleaved(grp, refine_iters)]
            re = _fleet_mean([times])[0]
            idx = {ks: i for i, ks in enumerate(todo)}
            for (ks, _, t), us in zip(cand, re):
                row = fleet[idx[ks]]
                row[t] = us
            # tiles not re-timed keep their (slower by > tol) phase-1 times
    for (ks, (key, _, _)), ts in zip(todo.items(), fleet):
        best = min(range(ntiles), key=lambda t: ts[t]) if ntiles else -1
        if ntiles and ts[best] == float("inf"):
            best = -1
        results[ks] = (best, round(ts[best], 2) if best >= 0 else None)
        if verbose:
            print(f"autotune {key} -> tile {best} {results[ks][1]} us", flush=True)
    # runner-up tiles per key (by the same timing), for the in-graph refine pass
    # (graph_refine below): every tile within ``ALT_TOL`` of the best, best first
    alts = {}
    for (ks, _), ts in zip(todo.items(), fleet):
        fin = sorted((ts[t], t) for t in range(ntiles) if ts[t] != float("inf"))
        if fin:
            alts[ks] = [t for us, t in fin if us <= fin[0][0] * (1.0 + ALT_TOL)][:1 + ALT_MAX]
    alts.update({k: v for k, v in cache_alts.items() if k not in alts})
    for layer, key, fn in rec:
        ks = repr(key)
        layer.tile = (results.get(ks) or cache[ks])[0]
        # runner-ups survive a warm restart (the cache keeps them), so the in-graph refine
        # can still work within its budget on a cache hit
        layer.tile_alts = alts.get(ks, [layer.tile])
        layer.tile_us = (results.get(ks) or cache[ks])[1] or 0.0
        if ks not in results:
            results[ks] = cache[ks]
    if cache_path and todo and parallel.info().local_rank == 0:  # one writer per VM disk
        cache.update(results)
        _write_cache(cache_path, sig, {k: [v[0], v[1], alts.get(k, [v[0]])]
                                       for k, v in cache.items()})
    return results


def _fleet_cache(cache: Dict, keys) -> Dict:
    """Data-parallel ranks use their tune caches only if EVERY rank has one covering
    ``keys`` and all hold the SAME picks: VMs that each tuned alone earlier would pin
    different tiles (split-K on one, not on the other) and break the bitwise replica check
    (C4).  One min and one max all-reduce of a digest of the picks; otherwise every rank
    drops its cache and re-tunes (identity when not distributed)."""
    from .. import parallel

    if not parallel.is_dist():
        return cache
    dg = _picks_digest(cache, keys) if cache else -1.0
    lo, = parallel.allreduce_scalars([dg], op="min")
    hi, = parallel.allreduce_scalars([dg], op="max")
    return cache if lo >= 0 and lo == hi else {}


def _picks_digest(cache: Dict, keys) -> float:
    """Order-independent digest of the picks for ``keys`` as an exact float (52 bits), for
    a min/max all-reduce agreement check across data-parallel ranks."""
    import hashlib

    doc = json.dumps(sorted((k, int(cache[k][0])) for k in set(keys) if k in cache))
    return float(int(hashlib.sha256(doc.encode()).hexdigest()[:13], 16))


def _write_cache(path: str, sig: str, picks: Dict) -> None:
    """Atomically (re)write the tune cache.  The in-graph refined tiles of earlier engines
    (other batches / stream counts) are kept while the signature still matches."""
    try:
        old = {}
        if os.path.exists(path):
            with open(path) as f:
                old = json.load(f)
        refined = old.get("refined", {}) if isinstance(old, dict) and old.get("signature") == sig else {}
        _dump_atomic(path, {"signature": sig, "picks": picks, "refined": refined})
    except (OSError, ValueError):
        pass  # read-only disk: tuning still applied, just not remembered


def _add_refined(path: str, key: str, rows) -> None:
    """Store graph_refine's per-layer tiles under ``key`` in an existing tune cache (whose
    picks the refined engine was tuned from); no cache file, nothing stored."""
    try:
        with open(path) as f:
            doc = json.load(f)
        if not isinstance(doc, dict) or "signature" not in doc:
            return
        doc.setdefault("refined", {})[key] = rows
        _dump_atomic(path, doc)
    except (OSError, ValueError):
        pass


def _dump_atomic(path: str, doc: Dict) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(doc, f, indent=0)
    os.replace(tmp, path)


ALT_TOL = 0.25  # runner-ups within 25 % of a layer's best (isolated timing) are graph-tested
ALT_MAX = 2     # ... at most two per layer


def graph_refine(engine, budget_s: float = 30.0, min_gain: float = 0.003,
                 verbose: bool = False, cache_path: str = None, ab=None) -> Dict:
    """In-graph tile refinement: the per-layer timing above measures a
    layer alone (or as concurrent copies of itself), but in the bench graph each kernel
    runs next to the previous and next layer of its own slice and whatever the other
    slice runs at that moment.  A tile that wins alone can lose there, and the reverse.

    For every layer with runner-up tiles (``layer.tile_alts``), largest layers first, the
    step graph is re-captured with the runner-up and timed against the current graph,
    replays interleaved A B B A ... on the same stream (drift hits both alike).  A change
    is kept only if the WHOLE STEP gets faster by more than ``min_gain`` in two separate
    measurements.  Stops at ``budget_s``.

    Verify before commit: when anything was kept, the refined graph is
    A/B-timed once more against the ORIGINAL capture; unless it wins by ``min_gain`` every
    layer's tile and the original graph are restored.  ``step_ms_before`` /
    ``step_ms_after`` come from that one interleaved measurement (original vs final; the
    same graph twice when nothing was kept).  Kept tiles go to ``cache_path`` (per layer
    ordinal, per batch x streams), so a warm restart reuses them.  ``ab``: timing hook
    (tests).  Returns {"trials", "kept", "reverted", "step_ms_before", "step_ms_after"}."""
    import time as _time

    ab = ab or _ab
    layers, order = [], []
    with record_convs() as rec:
        engine.model(engine.frames[:engine.batch // engine.n_streams])
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    seen = set()
    for layer, key, fn in rec:
        if id(layer) in seen:
            continue
        seen.add(id(layer))
        order.append((layer, repr(key)))
        if len(getattr(layer, "tile_alts", ())) >= 2:
            layers.append(layer)
    layers.sort(key=lambda l: -(getattr(l, "tile_us", 0.0) or 0.0))  # largest first
    if not layers or engine.graph is None:
        return {"trials": 0, "kept": 0, "reverted": False}
    t_end = _time.perf_counter() + budget_s
    orig, orig_out = engine.graph, engine.outputs
    orig_tiles = [(l, l.tile) for l, _ in order]
    cur, cur_out = orig, orig_out
    base = _replay_ms(cur, 3) if ab is _ab else 1.0
    rounds = max(4, min(40, int(200.0 / max(base, 1e-3))))
    trials = kept = 0
    from .. import parallel

    dist = parallel.is_dist()

    def fleet(gain, over):
        """Data-parallel ranks decide together (mean gain, any rank over budget): every
        replica must pin the same tiles (C4 compares their outputs)."""
        if not dist:
            return gain, over
        g, o = parallel.allreduce_scalars([gain, 1.0 if over else 0.0], op="sum")
        return g / parallel.info().world_size, o > 0

    for layer in layers:
        for t in layer.tile_alts:
            if t == layer.tile:
                continue
            if fleet(0.0, _time.perf_counter() > t_end)[1]:
                break
            old = layer.tile
            layer.tile = t
            g = None
            try:
                g, g_out = engine.capture()
                ok = 1.0
            except RuntimeError:  # tile not valid in this context
                ok = 0.0
            if fleet(ok, False)[0] < 1.0:  # invalid on some rank: skip everywhere
                layer.tile = old
                g = g_out = None
                continue
            trials += 1
            a, b = ab(cur, g, rounds)
            gain = fleet((a - b) / a, False)[0]
            if gain > min_gain:
                a2, b2 = ab(cur, g, 2 * rounds)
                gain = min(gain, fleet((a2 - b2) / a2, False)[0])
            if gain > min_gain:
                kept += 1
                if cur is not orig:
                    del cur, cur_out
                cur, cur_out = g, g_out
                if verbose:
                    print(f"graph_refine: tile {old} -> {t}: step {a:.3f} -> {b:.3f} ms",
                          flush=True)
            else:
                layer.tile = old
                del g, g_out
    # final check: the refined graph against the original capture, one interleaved A/B
    before, after = ab(orig, cur, 2 * rounds)
    reverted = False
    if kept:
        gain = fleet((before - after) / before, False)[0]
        if gain <= min_gain:  # the per-trial wins did not add up: keep the original
            reverted = True
            for l, t in orig_tiles:
                l.tile = t
            cur, cur_out = orig, orig_out
            after = before
    else:
        before = after = round((before + after) / 2, 4)  # one graph: no difference to report
    engine.graph, engine.outputs = cur, cur_out  # a rejected capture last set outputs
    if cache_path and kept and not reverted and parallel.info().local_rank == 0:
        # next to the per-key picks this engine was tuned from (same signature): a warm
        # restart of the same batch x streams re-applies them (apply_refined)
        _add_refined(cache_path, f"b{engine.batch}s{engine.n_streams}",
                     [[i, k, l.tile] for i, (l, k) in enumerate(order)])
    return {"trials": trials, "kept": 0 if reverted else kept, "reverted": reverted,
            "step_ms_before": round(before, 4), "step_ms_after": round(after, 4)}


def apply_refined(engine, cache_path: str) -> int:
    """Re-apply the in-graph refined tiles a previous engine of the same batch x streams
    stored in ``cache_path`` (graph_refine), layer by layer, when every layer's shape key
    still matches.  Returns the number of layers whose tile changed."""
    if not cache_path or not os.path.exists(cache_path):
        return 0
    try:
        with open(cache_path) as f:
            doc = json.load(f)
        rows = doc.get("refined", {}).get(f"b{engine.batch}s{engine.n_streams}")
    except (OSError, ValueError, AttributeError):
        return 0
    if not rows:
        return 0
    order = []
    with record_convs() as rec:
        engine.model(engine.frames[:engine.batch // engine.n_streams])
    seen = set()
    for layer, key, fn in rec:
        if id(layer) not in seen:
            seen.add(id(layer))
            order.append((layer, repr(key)))
    if len(rows) != len(order) or any(k != ok for (i, k, t), (_, ok) in zip(rows, order)):
        return 0
    n = 0
    for (i, k, t), (layer, _) in zip(rows, order):
        if layer.tile != t:
            layer.tile = int(t)
            n += 1
    return n


def _replay_ms(g, n: int) -> float:
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    st.record()
    for _ in range(n):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / n


def _ab(ga, gb, rounds: int):
    """Median ms per replay of graphs A and B, interleaved (A B, B A, A B ...)."""
    ta, tb = [], []
    _hold_gpu(2 * rounds)
    for r in range(rounds):
        order = ((ga, ta), (gb, tb)) if r % 2 == 0 else ((gb, tb), (ga, ta))
        for g, acc in order:
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            g.replay()
            en.record()
            acc.append((st, en))
    torch.cuda.synchronize()
    med = lambda xs: sorted(s.elapsed_time(e) for s, e in xs)[len(xs) // 2]  # noqa: E731
    return med(ta), med(tb)


def _cache_signature(ntiles: int, concurrency: int, world: int = 1) -> str:
    """Identity of what a cached pick depends on: the kernel library build (size and
    mtime of the loaded .so), its tile table (after KVEDGE_TILE_LIMIT), the device, the
    timing concurrency and the data-parallel world (fleet-mean picks vs a lone tune)."""
    from .. import ops

    try:
        st = os.stat(ops._LIB_PATH)
        lib = f"{st.st_size}:{int(st.st_mtime)}"
    except OSError:
        lib = "?"
    dev = torch.cuda.get_device_name() if torch.cuda.is_available() else "cpu"
    return f"lib={lib};tiles={ntiles};conc={concurrency};world={world};dev={dev}"
