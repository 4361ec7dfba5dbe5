#!/usr/bin/env python3
"""ISA lint for the gfx950 kernels: compile to assembly and report, per kernel, how many MFMAs
wait out a full LDS or memory round trip (an ``s_waitcnt lgkmcnt(0)`` / ``vmcnt(0)`` right in
front of them), VGPR / AGPR use and spills.

This is how round 4 found that hipcc had sunk every fragment read of the direct conv family
(conv_direct.hip) to just before its MFMA: 100 % of the MFMAs of every instantiation sat behind an
``lgkmcnt(0)`` although the source described a read ring (docs/kernels.md, "Direct family, round 4").

  python tools/isa_lint.py csrc/kernels/conv_direct.hip            # table
  python tools/isa_lint.py csrc/kernels/conv_direct.hip --max-lgkm0 0.1 --match conv3x3_direct
      # exit 1 if any matching kernel with >= 16 MFMAs has more than 10 % of them behind lgkmcnt(0)
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def compile_asm(src: str, out: str) -> None:
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-inline-asm",
           "-I" + os.path.join(ROOT, "csrc", "kernels"), "--cuda-device-only", "-S", src, "-o", out]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)


def _metadata(asm: str) -> dict:
    out = {}
    md = asm[asm.find("amdhsa.kernels:"):]
    for ent in re.split(r"\n  - ", md):
        name = re.search(r"\.name:\s+(\S+)", ent)
        if not name:
            continue
        get = lambda k: int(m.group(1)) if (m := re.search(re.escape(k) + r":\s*(\d+)", ent)) else 0  # noqa
        out[name.group(1)] = {"vgpr": get(".vgpr_count"), "agpr": get(".agpr_count"),
                              "spill": get(".vgpr_spill_count")}
    return out


def analyse(asm: str):
    """Yield (kernel, stats) for every kernel body in an assembly file."""
    meta = _metadata(asm)
    for m in re.finditer(r"^(_Z[^:\s]+):", asm, re.M):
        name = m.group(1)
        end = asm.find(".Lfunc_end", m.end())
        prev = None
        n_mfma = lgkm0 = vm0 = 0
        for line in asm[m.end():end].splitlines():
            t = line.strip()
            if not t or t.startswith((";", ".")):
                continue
            if t.startswith("v_mfma"):
                n_mfma += 1
                if prev and prev.startswith("s_waitcnt"):
                    lgkm0 += "lgkmcnt(0)" in prev
                    vm0 += "vmcnt(0)" in prev
            if not t.startswith("s_nop"):
                prev = t
        st = {"mfma": n_mfma, "lgkm0": lgkm0, "vm0": vm0}
        st.update(meta.get(name, {}))
        yield name, st


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="+")
    ap.add_argument("--match", default="", help="only kernels whose mangled name contains this")
    ap.add_argument("--max-lgkm0", type=float, default=None,
                    help="fail if a kernel with >= 16 MFMAs has more than this fraction of them "
                         "right behind an lgkmcnt(0)")
    ap.add_argument("--no-spill", action="store_true", help="fail on any VGPR spill")
    a = ap.parse_args(argv)
    bad = []
    print("| file | kernel | mfma | behind lgkmcnt(0) | behind vmcnt(0) | vgpr | agpr | spill |")
    print("|---|---|---|---|---|---|---|---|")
    with tempfile.TemporaryDirectory() as td:
        for src in a.sources:
            out = os.path.join(td, os.path.basename(src) + ".s")
            compile_asm(src, out)
            with open(out) as f:
                asm = f.read()
            for name, st in analyse(asm):
                if a.match and a.match not in name:
                    continue
                n = st["mfma"]
                fl = st["lgkm0"] / n if n else 0.0
                fv = st["vm0"] / n if n else 0.0
                print(f"| {os.path.basename(src)} | {name[:90]} | {n} | {fl:.0%} | {fv:.0%} | "
                      f"{st.get('vgpr', '?')} | {st.get('agpr', '?')} | {st.get('spill', '?')} |")
                if a.max_lgkm0 is not None and n >= 16 and fl > a.max_lgkm0:
                    bad.append((name, "lgkmcnt(0)", fl))
                if a.no_spill and st.get("spill", 0) > 0:
                    bad.append((name, "spill", st["spill"]))
    for name, what, v in bad:
        print(f"FAIL {what} {v}: {name}", file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
