"""The v6 N-loop kernel (csrc/kernels/conv_nloop.hip) synchronises every LDS read with an
exact, compile-time `s_waitcnt vmcnt(n)`; a count one too high would let a wave read a ring
slot before its DMA landed.  The library replays each instantiated tile's per-wave VMEM issue
order on the host and checks every wait the kernel uses against the exact count
(kv_nloop_sched_check).  Runs on the CPU: no GPU needed, only the built library."""
import pytest
import torch

from kvedge_amd import ops


def test_nloop_wait_schedule_is_safe():
    if not ops.load():
        pytest.skip("native library not built")
    rc = int(torch.ops.kvedge.nloop_sched_check())
    assert rc == 0, f"tile {rc // 10000}: schedule violation code {rc % 10000}"
