#!/bin/bash
# Three PMC passes (kernel-trace + counters only, each its own run) over any python probe.
# Usage: tools/pmc_cmd.sh <outdir> <python-script> [args...]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- \
    python3 "$@" > $OUT/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1 || true
echo done
