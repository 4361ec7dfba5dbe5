#!/bin/bash
# PMC passes (kernel-trace + counters only) over ONE layer/tile of tools/tile_probe.py.
# Usage: tools/pmc_layer.sh <layer> <tile> [outdir]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
L=${1:-s3.c2}; T=${2:-6}; OUT=${3:-gpurun_out/pmc_layer}
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- \
    python3 tools/tile_probe.py --only $L --tiles $T --iters 3 --batch ${PMC_BATCH:-256} > $OUT/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1 || true
echo done
