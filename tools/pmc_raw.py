#!/usr/bin/env python3
"""Raw counter values of one kernel from rocprofv3 --pmc passes: for each counter, the value
of the FASTEST dispatch whose name contains --match (one pass per directory p*/).

  python tools/pmc_raw.py gpurun_out/pmc_x --match conv_pp_kernel
"""
import argparse
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--match", required=True)
    a = ap.parse_args()
    out = {}
    for p in sorted(glob.glob(f"{a.root}/p*/*counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(p)) if a.match in r["Kernel_Name"]]
        disp = {}
        for r in rows:
            k = int(r["Dispatch_Id"])
            d = disp.setdefault(k, {"dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if not disp:
            continue
        best = min(disp.values(), key=lambda d: d["dur"])
        out.setdefault("dur_us", best["dur"] / 1e3)
        for k, v in best.items():
            if k != "dur":
                out[k] = v
    for k, v in out.items():
        print(f"{k:32s} {v:16.1f}")


if __name__ == "__main__":
    main()
