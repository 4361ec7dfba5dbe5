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


def _time(fn: Callable[[int], object], tile: int, iters: int) -> float:
    fn(tile)
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


def autotune(model: Callable, example_input: torch.Tensor, iters: int = 5,
             cache_path: str = None, verbose: bool = False) -> Dict:
    """Tune every conv of ``model`` for ``example_input``'s shape. Returns {key: (tile, us)}."""
    if not example_input.is_cuda:
        return {}
    cache = {}
    if cache_path and os.path.exists(cache_path):
        with open(cache_path) as f:
            cache = {k: tuple(v) for k, v in json.load(f).items()}
    with record_convs() as rec:
        model(example_input)
    torch.cuda.synchronize()
    ntiles = int(torch.ops.kvedge.conv_num_tiles())
    results: Dict = {}
    for layer, key, fn in rec:
        ks = repr(key)
        if ks in results or ks in cache:
            layer.tile = (results.get(ks) or cache[ks])[0]
            results.setdefault(ks, cache.get(ks))
            continue
        best, best_t = -1, float("inf")
        for t in range(ntiles):
            try:
                dt = _time(fn, t, iters)
            except RuntimeError:  # tile not valid for this layer kind
                continue
            if dt < best_t:
                best, best_t = t, dt
        layer.tile = best
        results[ks] = (best, round(best_t * 1e3, 2))
        if verbose:
            print(f"autotune {key} -> tile {best} {best_t * 1e3:.1f} us", flush=True)
    if cache_path:
        os.makedirs(os.path.dirname(cache_path) or ".", exist_ok=True)
        cache.update(results)
        with open(cache_path, "w") as f:
            json.dump(cache, f, indent=0)
    return results
