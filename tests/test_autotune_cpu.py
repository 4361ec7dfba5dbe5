"""CPU tests of the autotuner's bookkeeping: the in-graph refine's keep /
reject / invalid-tile / final-revert logic on stub graphs and timings, the refined tiles'
round trip through the tune cache, and the cache signature + pick-agreement rules."""
import json
import os

import pytest
import torch

from kvedge_amd.engine import autotune as at
from kvedge_amd.models.layers import _record, _recorder_active


class _Layer:
    def __init__(self, name, tile, alts, us):
        self.name, self.tile, self.tile_alts, self.tile_us = name, tile, alts, us


class _Graph:
    def __init__(self, tiles):
        self.tiles = tiles


class _Engine:
    """What graph_refine touches: model (records its layers), frames, batch, n_streams,
    graph / outputs, capture()."""

    def __init__(self, layers, invalid=()):
        self.layers = layers
        self.invalid = set(invalid)
        self.frames = torch.zeros(4, 1)
        self.batch, self.n_streams = 4, 2
        self.captures = 0
        self.graph, self.outputs = self._snap(), object()

    def _snap(self):
        return _Graph(tuple(l.tile for l in self.layers))

    def model(self, x):
        if _recorder_active():
            for l in self.layers:
                _record(l, ("conv", l.name), None)

    def capture(self):
        if any(l.tile in self.invalid for l in self.layers):
            raise RuntimeError("tile not valid here")
        self.captures += 1
        return self._snap(), object()


def _cost_ab(cost, trial_bias=None):
    """Timing hook: a graph's step time is the sum of its layers' per-tile costs.
    ``trial_bias(tiles)`` (optional) is subtracted only while trials run -- a noisy
    measurement that makes a swap look better than it is, so the final check must catch it."""
    state = {"final": False}

    def ab(ga, gb, rounds):
        def t(g):
            v = sum(cost[i][tile] for i, tile in enumerate(g.tiles))
            if trial_bias and not state["final"]:
                v -= trial_bias(g.tiles)
            return v
        return t(ga), t(gb)
    return ab, state


def test_graph_refine_keeps_a_real_gain_and_persists_it(tmp_path):
    a = _Layer("a", 0, [0, 1], 100.0)
    b = _Layer("b", 5, [5, 6], 50.0)
    eng = _Engine([a, b])
    cost = [{0: 10.0, 1: 9.0}, {5: 4.0, 6: 4.5}]  # a: tile 1 is 10 % faster; b: 6 slower
    ab, _ = _cost_ab(cost)
    cache = tmp_path / "tune.json"
    cache.write_text(json.dumps({"signature": "sig", "picks": {}}))
    orig = eng.graph
    r = at.graph_refine(eng, budget_s=60, ab=ab, cache_path=str(cache))
    assert r["trials"] == 2 and r["kept"] == 1 and not r["reverted"]
    assert a.tile == 1 and b.tile == 5
    assert eng.graph is not orig and eng.graph.tiles == (1, 5)
    assert r["step_ms_before"] == 14.0 and r["step_ms_after"] == 13.0
    doc = json.loads(cache.read_text())
    assert doc["refined"]["b4s2"] == [[0, repr(("conv", "a")), 1], [1, repr(("conv", "b")), 5]]
    # a warm restart re-applies the refined tile layer by layer
    a2, b2 = _Layer("a", 0, [0], 100.0), _Layer("b", 5, [5], 50.0)
    eng2 = _Engine([a2, b2])
    assert at.apply_refined(eng2, str(cache)) == 1 and a2.tile == 1 and b2.tile == 5
    # ... but not onto a different network (shape keys differ)
    c3 = _Layer("c", 0, [0], 1.0)
    assert at.apply_refined(_Engine([c3, _Layer("b", 5, [5], 1.0)]), str(cache)) == 0
    assert c3.tile == 0


def test_graph_refine_rejects_slower_and_invalid_tiles():
    a = _Layer("a", 0, [0, 1, 2], 100.0)
    eng = _Engine([a], invalid={2})
    ab, _ = _cost_ab([{0: 10.0, 1: 10.5, 2: 1.0}])
    orig = eng.graph
    r = at.graph_refine(eng, budget_s=60, ab=ab)
    assert r["trials"] == 1 and r["kept"] == 0 and not r["reverted"]  # tile 2: no capture
    assert a.tile == 0 and eng.graph is orig
    assert r["step_ms_before"] == r["step_ms_after"] == 10.0


def test_graph_refine_reverts_when_final_ab_shows_no_gain():
    """per-trial wins that do not hold against the original capture
    (here: a biased trial measurement) are undone -- tiles and graph both."""
    a = _Layer("a", 0, [0, 1], 100.0)
    b = _Layer("b", 5, [5, 6], 50.0)
    eng = _Engine([a, b])
    cost = [{0: 10.0, 1: 10.02}, {5: 4.0, 6: 4.03}]  # both swaps are really slower
    ab, state = _cost_ab(cost, trial_bias=lambda tiles: 0.2 * (tiles[0] == 1) + 0.2 * (tiles[1] == 6))
    orig = eng.graph

    real = at._ab

    def ab_final_aware(ga, gb, rounds):
        # the final check is the only call comparing the ORIGINAL graph with the final one
        state["final"] = ga is orig and gb.tiles == (1, 6)
        return ab(ga, gb, rounds)
    try:
        r = at.graph_refine(eng, budget_s=60, ab=ab_final_aware)
    finally:
        assert at._ab is real
    assert r["kept"] == 0 and r["reverted"] is True
    assert a.tile == 0 and b.tile == 5 and eng.graph is orig
    assert r["step_ms_after"] == r["step_ms_before"]


def test_cache_signature_includes_world_and_tile_limit(monkeypatch, tmp_path):
    """a KVEDGE_TILE_LIMIT run and a full run, or a lone tune and a fleet-mean
    tune, never share cached picks."""
    monkeypatch.setattr(at.torch.cuda, "is_available", lambda: False)
    s_full = at._cache_signature(120, 2, 1)
    assert s_full != at._cache_signature(100, 2, 1)
    assert s_full != at._cache_signature(120, 2, 8)
    assert "world=8" in at._cache_signature(120, 2, 8)


def test_picks_digest_agreement_rule():
    keys = ["k1", "k2", "k3"]
    a = {"k1": (3, 1.0), "k2": (7, 2.0), "k3": (9, 3.0)}
    b = dict(a, k2=(8, 2.0))
    assert at._picks_digest(a, keys) == at._picks_digest(dict(reversed(list(a.items()))), keys)
    assert at._picks_digest(a, keys) != at._picks_digest(b, keys)
    d = at._picks_digest(a, keys)
    assert d == float(int(d)) and 0 <= d < 2 ** 53  # exact through a float all-reduce


def test_write_cache_keeps_refined_only_for_the_same_signature(tmp_path):
    p = str(tmp_path / "c.json")
    at._write_cache(p, "s1", {"k": [1, 2.0, [1, 3]]})
    at._add_refined(p, "b64s1", [[0, "k", 3]])
    at._write_cache(p, "s1", {"k": [1, 2.0, [1, 3]], "k2": [0, 1.0, [0]]})
    doc = json.loads(open(p).read())
    assert doc["refined"] == {"b64s1": [[0, "k", 3]]} and "k2" in doc["picks"]
    at._write_cache(p, "s2", {"k": [2, 2.0, [2]]})  # new library: old refinements dropped
    assert json.loads(open(p).read())["refined"] == {}
    assert not os.path.exists(p + ".tmp")


def _fleet_worker(rank, world, port, caches, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from kvedge_amd import parallel

    parallel.init_from_env(prefer_gpu=False)
    try:
        out = [at._fleet_cache(c[rank], ["k1", "k2"]) for c in caches]
        q.put((rank, out))
    finally:
        parallel.shutdown()


def test_dist_cache_agreement_gloo():
    """two ranks whose caches hold different picks both re-tune (empty
    cache on every rank); equal picks are kept; a rank without a cache makes all re-tune."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    same = {"k1": (3, 1.0), "k2": (4, 2.0)}
    caches = [
        [same, dict(same)],                               # agree -> kept
        [same, {"k1": (3, 1.0), "k2": (5, 2.0)}],         # k2 differs -> dropped
        [same, {}],                                       # one rank has none -> dropped
    ]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_fleet_worker, args=(r, 2, port, caches, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        kept, differ, missing = res[r]
        assert kept == caches[0][r] and differ == {} and missing == {}


def test_splitk_tile_range_from_native():
    """ops.is_splitk() must cover exactly the native split-K family: it decides which tiles
    get an fp32 slab workspace, and a derived base once drifted when a family was appended."""
    from kvedge_amd import ops
    if not ops.load():
        pytest.skip("native library not built")
    import torch
    base = int(torch.ops.kvedge.conv_splitk_base())
    assert ops.SPLITK0 == base
    assert ops.is_splitk(base) and ops.is_splitk(base + ops.N_SPLITK_TILES - 1)
    assert not ops.is_splitk(base - 1) and not ops.is_splitk(base + ops.N_SPLITK_TILES)
    # split-K, direct-epilogue, skinny and v14 families follow in that order
    assert base + ops.N_SPLITK_TILES + ops.N_DE_TILES + ops.N_SKINNY_TILES + 4 == \
        int(torch.ops.kvedge.conv_num_tiles())
