#!/usr/bin/env python3
"""Per-call kernel list of ONE measured step from a profile_forward.py kernel trace."""
import csv
import sys

path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = max(i for i, r in enumerate(rows) if "synth_kernel" in r["Kernel_Name"]
          and "dev" not in r["Kernel_Name"])
body = rows[idx + 1:]
if n == 0:  # one step = up to the second synth_dev_kernel
    starts = [i for i, r in enumerate(body) if "synth_dev_kernel" in r["Kernel_Name"]]
    n = starts[1] if len(starts) > 1 else len(body)
tot = 0.0
for r in body[:n]:
    name = r["Kernel_Name"].replace("void ", "").replace("kvedge::(anonymous namespace)::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f"{d:8.1f} {r.get('Grid_Size_X', ''):>9} {name.split('(')[0][:64]}")
print(f"total {tot:.1f} us over {n} kernels")
