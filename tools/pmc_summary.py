#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs: per (kernel, grid) the FASTEST dispatch's counters,
plus derived metrics (achieved HBM GB/s, VALU/MFMA per wave, wait fraction)."""
import collections
import csv
import glob
import sys


def load(path):
    d = collections.defaultdict(dict)
    meta = {}
    rows = list(csv.DictReader(open(path)))
    # tools/profile_forward.py marks the measured region with a non-graph synth_kernel:
    # keep only the dispatches after it (autotune / warm-up noise excluded)
    marks = [int(r["Dispatch_Id"]) for r in rows if "synth_kernel" in r["Kernel_Name"]
             and "synth_dev" not in r["Kernel_Name"]]
    first = max(marks) if marks else -1
    for r in rows:
        k = int(r["Dispatch_Id"])
        if k <= first:
            continue
        d[k][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["End_Timestamp"]) -
                   int(r["Start_Timestamp"]), int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]),
                   int(r["LDS_Block_Size"]))
    return d, meta


def main(root="gpurun_out/pmc", top=40, pattern="p*/p*_counter_collection.csv"):
    groups = collections.defaultdict(dict)
    for p in sorted(glob.glob(f"{root}/{pattern}")):
        d, meta = load(p)
        for k, cs in d.items():
            name, grid, dur, vg, ag, lds = meta[k]
            key = (name, grid)
            best = groups[key].get(p)
            if best is None or dur < best[0]:
                groups[key][p] = (dur, cs, vg, ag, lds)
    rows = []
    for (name, grid), per in groups.items():
        cs = {}
        dur = min(v[0] for v in per.values())
        vg = ag = lds = 0
        for v in per.values():
            cs.update(v[1])
            vg, ag, lds = v[2], v[3], v[4]
        short = name.replace("void kvedge::(anonymous namespace)::", "").split("(")[0]
        waves = cs.get("SQ_WAVES", 0) or 1
        r = {"kernel": short[:48], "grid": grid, "us": dur / 1e3, "vgpr": vg, "agpr": ag, "lds": lds,
             # FETCH_SIZE = TCC_EA0_RDREQ x 64 B and reads 1/2 of a wide streaming read on
             # gfx950 (MI355X_MICROARCH.md "HBM"): bytes read ~ 128 B x RDREQ; writes 64 B each
             "rd_MB": 128 * cs.get("TCC_EA0_RDREQ_sum", 0) / 1e6,
             "wr_MB": 64 * cs.get("TCC_EA0_WRREQ_sum", 0) / 1e6,
             "rd_GBs": 128 * cs.get("TCC_EA0_RDREQ_sum", 0) / max(dur, 1),
             "wr_GBs": 64 * cs.get("TCC_EA0_WRREQ_sum", 0) / max(dur, 1),
             "valu/w": cs.get("SQ_INSTS_VALU", 0) / waves, "mfma/w": cs.get("SQ_INSTS_MFMA", 0) / waves,
             "lds/w": cs.get("SQ_INSTS_LDS", 0) / waves,
             "wait%": 100 * cs.get("SQ_WAIT_ANY", 0) / max(cs.get("SQ_WAVE_CYCLES", 1), 1),
             "winst%": 100 * cs.get("SQ_WAIT_INST_ANY", 0) / max(cs.get("SQ_WAVE_CYCLES", 1), 1),
             # busy cycles over SIMD-cycles (GUI_ACTIVE is summed over the 8 XCDs; 256 CUs x
             # 4 SIMDs); "n/a" when the pass did not collect both counters (round-4 tables
             # printed 0.0 there, which read as "MFMA idle")
             "mfma_busy%": (100 * cs["SQ_VALU_MFMA_BUSY_CYCLES"] /
                            max(cs["GRBM_GUI_ACTIVE"] / 8 * 256 * 4, 1))
                           if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs
                           else "n/a",
             "l2hit%": 100 * cs.get("TCC_HIT_sum", 0) /
                       max(cs.get("TCC_HIT_sum", 0) + cs.get("TCC_MISS_sum", 0), 1),
             "bankc": cs.get("SQ_LDS_BANK_CONFLICT", 0),
             "clk_GHz": cs.get("GRBM_GUI_ACTIVE", 0) / 8 / max(dur, 1)}
        rows.append(r)
    rows.sort(key=lambda r: -r["us"])
    cols = list(rows[0].keys()) if rows else []
    print("| " + " | ".join(cols) + " |")
    print("|" + "---|" * len(cols))
    for r in rows[:top]:
        print("| " + " | ".join(f"{v:.1f}" if isinstance(v, float) else str(v) for v in r.values()) + " |")


if __name__ == "__main__":
    main(*(sys.argv[1:2] or []), *([40, sys.argv[2]] if len(sys.argv) > 2 else []))
