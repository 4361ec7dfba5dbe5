# Round 5 (q): fused C2f standalone timing by strip height; PMC of the kernel
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5q}
timeout -k 10 300 python -u tools/c2f_probe.py --batch 256 --strips 40,20,8,4 > gpurun_out/${T}_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_probe.txt; exit 1; }
cat gpurun_out/${T}_probe.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/${T}_pmc1 -o p -- python3 tools/c2f_probe.py --batch 256 --strips 40 --iters 2 > gpurun_out/${T}_pmc1.log 2>&1 || { tail -5 gpurun_out/${T}_pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/${T}_pmc2 -o p -- python3 tools/c2f_probe.py --batch 256 --strips 40 --iters 2 > gpurun_out/${T}_pmc2.log 2>&1 || { tail -5 gpurun_out/${T}_pmc2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("r5q_pmc1", "r5q_pmc2"):
    for f in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(float); n = collections.Counter()
        for r in csv.DictReader(open(f)):
            if "c2f16" not in r.get("Kernel_Name", ""): continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
        print(d, {k: round(v / max(n[k], 1)) for k, v in agg.items()})
PY
rm -rf gpurun_out/${T}_pmc1 gpurun_out/${T}_pmc2
