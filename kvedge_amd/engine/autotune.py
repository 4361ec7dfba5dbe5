"""Per-layer tile autotuner for the implicit-GEMM conv kernel.

One instrumented eager forward records every conv call with its live tensors; each
distinct call shape is then timed with every tile of the kernel's tile table on
those exact tensors (HIP events, median of a few launches) and the fastest tile is
pinned on the DeployedConv before hipGraph capture.  Correctness never depends on
the tile: all tiles compute the same result (tests/test_kernels_gpu.py
test_conv_every_tile).
"""
from __future__ import annotations

import json
import os
from typing import Callable, Dict, Tuple

import torch

from .. import ops
from ..models.layers import record_convs


def _key(conv, a) -> Tuple:
    s = conv.spec
    return (s.cin, s.cout, s.kh, s.kw, s.stride, s.pad, s.act, s.mode, tuple(a["x"].shape),
            a["x_coff"], tuple(a["out"].shape), a["res"] is not None)


def _time_call(conv, a, tile: int, iters: int) -> float:
    fn = lambda: ops.conv2d(a["x"], conv.spec, conv.w, conv.b, res=a["res"], out=a["out"],  # noqa: E731
                            x_coff=a["x_coff"], y_coff=a["y_coff"], r_coff=a["r_coff"],
                            tile=tile)
    fn()
    evs = []
    for _ in range(iters):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        fn()
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
    for conv, a in rec:
        k = _key(conv, a)
        ks = repr(k)
        if ks in results:
            conv.tile = results[ks][0]
            continue
        if ks in cache:
            results[ks] = cache[ks]
            conv.tile = cache[ks][0]
            continue
        best, best_t = -1, float("inf")
        for t in range(ntiles):
            dt = _time_call(conv, a, t, iters)
            if dt < best_t:
                best, best_t = t, dt
        conv.tile = best
        results[ks] = (best, round(best_t * 1e3, 2))
        if verbose:
            print(f"autotune {k} -> tile {best} {best_t * 1e3:.1f} us", flush=True)
    if cache_path:
        os.makedirs(os.path.dirname(cache_path) or ".", exist_ok=True)
        cache.update(results)
        with open(cache_path, "w") as f:
            json.dump(cache, f, indent=0)
    return results
