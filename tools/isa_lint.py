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
        st = {"mfma": n_mfma, "lgkm0": lgkm0, "vm0": vm0,
              "inflight": inflight_hazards(asm, m.end(), end)}
        st.update(meta.get(name, {}))
        yield name, st


# --------------------------------------------------------------------------- in-flight check
# The asm loads of common.h (lds_read16 / vm_load16, and conv_seam.hip's residual loads) are
# invisible to hipcc's wait-count pass: their destination registers are written when the data
# returns, after the asm statement.  The contract is that nothing touches those registers until
# the counted s_waitcnt that retires the load.  A compiler copy of such a register (a v_mov at
# a loop back-edge, a spill, a re-materialised value) before that wait reads garbage: that is
# how round 4's YOLO stem2 prefetch (commit ad7a357) produced NaNs at 640x640.  This pass walks
# each kernel's ISA with the two counters modelled:
#   * lgkmcnt: LDS ops complete in order among themselves (SMEM ops may complete out of order,
#     but counter <= N still means at most N LDS ops are outstanding), so a wait
#     ``lgkmcnt(N)`` retires every LDS op but the N youngest;
#   * vmcnt: vector-memory ops (loads, stores, LDS DMA) retire in issue order: ``vmcnt(N)``
#     retires all but the N youngest;
# and reports every instruction that reads or writes a VGPR of an asm-issued load that is
# still in flight.  Branches are followed with the in-flight state (each edge once), so a
# value carried around a loop back-edge is checked on the next trip through the header.
_VREG = re.compile(r"(?<![\w\[])v\[(\d+):(\d+)\]|(?<![\w\[])v(\d+)\b")
_LABEL = re.compile(r"^(\.L\w+|\w+):")


def _vregs(operands: str):
    out = set()
    for m in _VREG.finditer(operands):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _body(asm: str, start: int, end: int):
    """[(kind, text, in_asm)] of one kernel: kind 'label' | 'ins'."""
    out, in_asm = [], False
    for line in asm[start:end].splitlines():
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        t = t.split(";", 1)[0].strip()
        if not t or t.startswith("."):
            if t and _LABEL.match(t):
                out.append(("label", _LABEL.match(t).group(1), in_asm))
            continue
        m = _LABEL.match(t)
        if m and t.endswith(":"):
            out.append(("label", m.group(1), in_asm))
            continue
        out.append(("ins", t, in_asm))
    return out


def _classify(ins: str):
    """-> ('lgkm'|'vm'|'smem'|None, is_load_with_vgpr_dest)"""
    op = ins.split()[0]
    if op.startswith("ds_"):
        return "lgkm", op.startswith("ds_read") or op.startswith("ds_load")
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime")):
        return "smem", False
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        is_load = ("load" in op) and not re.search(r"\blds\b", ins)
        return "vm", is_load
    return None, False


def inflight_hazards(asm: str, start: int, end: int, max_visits: int = 4):
    """[(instruction, asm load it touches)] for one kernel body (see the block comment)."""
    body = _body(asm, start, end)
    labels = {t: i for i, (k, t, _) in enumerate(body) if k == "label"}
    hazards = {}
    seen_edges = {}

    def walk(i, lgkm, vm):
        while i < len(body):
            kind, ins, in_asm = body[i]
            i += 1
            if kind == "label":
                continue
            op = ins.split()[0]
            if op == "s_waitcnt":
                m = re.search(r"lgkmcnt\((\d+)\)", ins)
                if m:
                    n = int(m.group(1))
                    lgkm = lgkm[len(lgkm) - n:] if n < len(lgkm) else lgkm
                    if n == 0:
                        lgkm = []
                m = re.search(r"vmcnt\((\d+)\)", ins)
                if m:
                    n = int(m.group(1))
                    vm = vm[len(vm) - n:] if 0 < n < len(vm) else ([] if n == 0 else vm)
                continue
            if op == "s_endpgm":
                return
            operands = ins[len(op):]
            regs = _vregs(operands)
            cls, is_load = _classify(ins)
            dest = set()
            if cls in ("lgkm", "vm") and is_load:
                first = operands.split(",")[0]
                dest = _vregs(first)
            # a later load of the same counter writing the same registers is not a hazard:
            # loads of one counter return in order, so the younger value lands last; its
            # address operands still must not read an in-flight register
            srcs = regs - dest if (cls in ("lgkm", "vm") and is_load) else regs
            for e, ecls in [(e, "lgkm") for e in lgkm] + [(e, "vm") for e in vm]:
                if not e[0]:
                    continue
                touch = (srcs if ecls == cls else regs) & e[0]
                if touch:
                    hazards.setdefault((i - 1, ins), e[1])
            if cls == "lgkm":
                lgkm = lgkm + [(dest if in_asm else set(), ins)]
            elif cls == "vm":
                vm = vm + [(dest if in_asm else set(), ins)]
            if op.startswith(("s_branch", "s_cbranch")) and not op.startswith("s_cbranch_g"):
                tgt = ins.split()[-1]
                live = any(e[0] for e in lgkm + vm)
                if tgt in labels and live:
                    key = (i - 1, tgt)
                    seen_edges[key] = seen_edges.get(key, 0) + 1
                    if seen_edges[key] <= max_visits:
                        walk(labels[tgt] + 1, list(lgkm), list(vm))
                if op == "s_branch":
                    # no fall-through: what follows is reached from another branch, whose
                    # in-flight loads that walk covers; scan it from an empty state
                    lgkm, vm = [], []

    walk(0, [], [])
    return [(body[k][1], src) for (k, _), src in sorted(hazards.items())]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="+")
    ap.add_argument("--match", default="", help="only kernels whose mangled name contains this")
    ap.add_argument("--max-lgkm0", type=float, default=None,
                    help="fail if a kernel with >= 16 MFMAs has more than this fraction of them "
                         "right behind an lgkmcnt(0)")
    ap.add_argument("--no-spill", action="store_true", help="fail on any VGPR spill")
    ap.add_argument("--inflight", action="store_true",
                    help="fail if any instruction touches a VGPR of an asm-issued load before "
                         "the s_waitcnt that retires it (the lds_read16 / vm_load16 contract)")
    a = ap.parse_args(argv)
    bad = []
    print("| file | kernel | mfma | behind lgkmcnt(0) | behind vmcnt(0) | vgpr | agpr | spill "
          "| in-flight reads |")
    print("|---|---|---|---|---|---|---|---|---|")
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
                hz = st["inflight"]
                print(f"| {os.path.basename(src)} | {name[:90]} | {n} | {fl:.0%} | {fv:.0%} | "
                      f"{st.get('vgpr', '?')} | {st.get('agpr', '?')} | {st.get('spill', '?')} "
                      f"| {len(hz)} |")
                if a.inflight and hz:
                    for ins, load in hz[:5]:
                        print(f"  in-flight: `{ins}` touches the destination of `{load}`",
                              file=sys.stderr)
                    bad.append((name, "in-flight register read", len(hz)))
                if a.max_lgkm0 is not None and n >= 16 and fl > a.max_lgkm0:
                    bad.append((name, "lgkmcnt(0)", fl))
                if a.no_spill and st.get("spill", 0) > 0:
                    bad.append((name, "spill", st["spill"]))
    for name, what, v in bad:
        print(f"FAIL {what} {v}: {name}", file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
