"""ISA regression guard (CPU; hipcc cross-compiles gfx950 here): the direct conv family's
fragment reads must stay a ring -- no more than 10 % of any instantiation's MFMAs right behind an
``s_waitcnt lgkmcnt(0)`` -- and no instantiation may spill.  Before round 4 hipcc sank every read
to its MFMA (100 % behind lgkmcnt(0)) and nothing noticed (tools/isa_lint.py)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="no hipcc")
def test_direct_conv_fragment_ring_and_no_spills():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_lint.py"),
                        os.path.join(ROOT, "csrc", "kernels", "conv_direct.hip"),
                        "--match", "conv3x3_direct", "--max-lgkm0", "0.1", "--no-spill"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:] + r.stdout[-2000:]
    rows = [l for l in r.stdout.splitlines() if "conv3x3_direct" in l]
    assert len(rows) >= 40, len(rows)  # every instantiation was analysed
