"""T-dist: data-parallel runtime with world_size 2/4 on CPU (gloo), one process per rank."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from kvedge_amd import parallel

    di = parallel.init_from_env(prefer_gpu=False)
    try:
        assert di.backend == "gloo" and di.world_size == world
        # C1: weights differ per rank before, equal after broadcast (multi-bucket)
        ts = [torch.full((1000,), float(rank)), torch.full((7, 3), 10.0 + rank),
              torch.full((5,), rank, dtype=torch.int32)]
        n = parallel.broadcast_tensors(ts, src=0, bucket_bytes=2048)
        ok_b = all(bool((t == t.flatten()[0]).all()) for t in ts) and ts[0][0] == 0 and \
            ts[1][0, 0] == 10.0 and int(ts[2][0]) == 0 and n >= 2
        # C2/C3
        s = parallel.allreduce_scalars([1.0, rank], op="sum")
        m = parallel.allreduce_scalars([rank * 1.5], op="max")
        g = parallel.all_gather_scalar(float(rank))
        # fleet autotune: per-tile timings averaged over ranks, invalid tiles stay inf
        from kvedge_amd.engine.autotune import _fleet_mean

        inf = float("inf")
        fm = _fleet_mean([[1.0 + rank, inf, 3.0], [inf, 2.0 * (rank + 1), 0.5]])
        parallel.barrier()
        q.put((rank, ok_b, s, m, g, fm))
    finally:
        parallel.shutdown()


@pytest.mark.parametrize("world", [2, 4])
def test_dp_collectives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_b, s, m, g, fm in res:
        assert ok_b
        mean_r = sum(range(world)) / world
        assert fm == [[1.0 + mean_r, float("inf"), 3.0], [float("inf"), 2.0 * (mean_r + 1), 0.5]]
        assert s == [float(world), float(sum(range(world)))]
        assert m == [1.5 * (world - 1)]
        assert g == [float(r) for r in range(world)]


def test_single_process_noop():
    from kvedge_amd import parallel

    os.environ.pop("WORLD_SIZE", None)
    di = parallel.init_from_env(prefer_gpu=False)
    assert di.world_size == 1 and not parallel.is_dist()
    assert parallel.broadcast_tensors([torch.ones(3)]) == 0
    assert parallel.allreduce_scalars([2.0]) == [2.0]
    assert parallel.all_gather_scalar(3.0) == [3.0]


def test_autotune_near_ties():
    from kvedge_amd.engine.autotune import _near_ties

    inf = float("inf")
    rows = [[10.0, 10.4, 12.0, inf], [5.0, 9.0, inf, inf], [inf, inf, inf, inf], [],
            [20.0, 20.0, 20.9, 21.5]]
    assert _near_ties(rows, 0.05) == [(0, 0), (0, 1), (4, 0), (4, 1), (4, 2)]
    assert _near_ties(rows, 0.0) == [(4, 0), (4, 1)]
