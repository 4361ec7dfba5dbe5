#!/bin/bash
# PMC counters for the ResNet-50 conv layers (separate passes; counters only with
# --kernel-trace/--stats, never with trace domains -- see gpurun rules).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
B=${1:-256}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p1 \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA \
  -- python3 tools/layer_bench.py --batch $B --iters 2 --no-torch --out $OUT/lb1.md > $OUT/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p2 \
  --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS \
  -- python3 tools/layer_bench.py --batch $B --iters 2 --no-torch --out $OUT/lb2.md > $OUT/p2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o p3 \
  --pmc WRITE_SIZE GRBM_GUI_ACTIVE \
  -- python3 tools/layer_bench.py --batch $B --iters 2 --no-torch --out $OUT/lb3.md > $OUT/p3.log 2>&1 || exit $?
echo done
