"""ISA regression guard (CPU; hipcc cross-compiles gfx950 here): the direct conv family's
fragment reads must stay a ring -- no more than 10 % of any instantiation's MFMAs right behind an
``s_waitcnt lgkmcnt(0)`` -- and no instantiation may spill.  Before round 4 hipcc sank every read
to its MFMA (100 % behind lgkmcnt(0)) and nothing noticed (tools/isa_lint.py).

The asm-ring contract (common.h lds_read16 / vm_load16, conv_seam.hip's residual loads) is a
checked invariant too: no instruction may read or write a destination VGPR of an asm-issued load
before the s_waitcnt that retires it (tools/isa_lint.py --inflight).  The check must flag the
round-4 YOLO stem2 prefetch (commit ad7a357, NaNs at 640x640: a back-edge v_mov copied the next
block's fragments while their ds_read_b128 was still in flight) and pass every kernel at HEAD."""
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
                        "--match", "conv3x3_direct", "--max-lgkm0", "0.1", "--no-spill",
                        "--inflight"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:] + r.stdout[-2000:]
    rows = [l for l in r.stdout.splitlines() if "conv3x3_direct" in l]
    assert len(rows) >= 40, len(rows)  # every instantiation was analysed


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="no hipcc")
def test_inflight_asm_loads_flag_ad7a357_and_pass_head():
    lint = os.path.join(ROOT, "tools", "isa_lint.py")
    bad = subprocess.run([sys.executable, lint, "--inflight",
                          os.path.join(ROOT, "tests", "fixtures", "yolo_stem2_ad7a357.hip")],
                         capture_output=True, text=True, timeout=900)
    assert bad.returncode == 1, bad.stdout + bad.stderr
    assert "in-flight" in bad.stderr and "v_mov" in bad.stderr  # the back-edge copies
    k = os.path.join(ROOT, "csrc", "kernels")
    ok = subprocess.run([sys.executable, lint, "--inflight", os.path.join(k, "conv_seam.hip"),
                         os.path.join(k, "yolo_stem2.hip"), os.path.join(k, "stem12.hip")],
                        capture_output=True, text=True, timeout=900)
    assert ok.returncode == 0, ok.stderr[-2000:]
    rows = [l for l in ok.stdout.splitlines() if l.startswith("| conv_seam")]
    assert len(rows) >= 8 and all(l.rstrip(" |").endswith("| 0") for l in rows)


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="no hipcc")
def test_round5_kernels_no_spill_no_inflight_reads():
    """The v12 edge-batch family (LDS-DMA rings behind asm waits) and the v13 fused C2f
    kernel (3 waves per SIMD at <= 168 VGPRs): every instantiation spill-free, and no read of
    an asm load's destination before its wait."""
    k = os.path.join(ROOT, "csrc", "kernels")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_lint.py"),
                        os.path.join(k, "conv_skinny.hip"), os.path.join(k, "c2f_fused.hip"),
                        "--no-spill", "--inflight"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:] + r.stdout[-2000:]
    rows = [l for l in r.stdout.splitlines() if l.startswith(("| conv_skinny", "| c2f_fused"))]
    assert len(rows) == 27 + 2, len(rows)  # 9 tiles x 3 modes, 2 widths
