#!/bin/bash
# PMC counter passes over one layer/tile of tools/tile_probe.py plus torch copy/fill
# (memory-system comparison).  Usage: tools/pmc_probe.sh <layer> <tile>
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_probe
mkdir -p $OUT
L=${1:-s1.c3-nores}; T=${2:-23}
i=0
for grp in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_WRITE_sum TCC_READ_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM" \
           "TA_BUFFER_WRITE_WAVEFRONTS_sum TA_BUFFER_COALESCED_WRITE_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT -o p$i -- \
    python3 tools/tile_probe.py --only $L --tiles $T --iters 3 > $OUT/p$i.log 2>&1 || exit $?
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT -o t$i -- \
    python3 tools/roofline_probe.py --bw-only > $OUT/t$i.log 2>&1 || exit $?
done
echo done
