#!/usr/bin/env python3
"""RCCL collective bandwidth through torch.distributed (one process per GPU / per VM).

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/allreduce_bench.py
Works with gloo on CPU too (tests).  Prints JSON lines (rank 0): algBW/busBW per size,
the same definitions as csrc/comm/rccl_bench.cpp."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-bytes", type=int, default=1 << 10)
    ap.add_argument("--max-bytes", type=int, default=1 << 28)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist

    from kvedge_amd import parallel

    di = parallel.init_from_env(prefer_gpu=True)
    n = di.world_size
    res = []
    b = a.min_bytes
    while b <= a.max_bytes:
        count = max(n, b // 2)
        x = torch.ones(count, dtype=torch.bfloat16, device=di.device)
        for _ in range(2):
            if n > 1:
                dist.all_reduce(x)
        if di.device.type == "cuda":
            torch.cuda.synchronize()
        parallel.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            if n > 1:
                dist.all_reduce(x)
        if di.device.type == "cuda":
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        (dt,) = parallel.allreduce_scalars([dt], op="max")
        alg = count * 2 / dt / 1e9
        r = {"coll": "all_reduce", "n": n, "bytes": count * 2, "us": round(dt * 1e6, 2),
             "algbw_GBps": round(alg, 3), "busbw_GBps": round(alg * 2 * (n - 1) / n, 3),
             "backend": di.backend}
        res.append(r)
        if di.is_main:
            print(json.dumps(r), flush=True)
        b *= 4
    parallel.shutdown()
    return res


if __name__ == "__main__":
    main()
