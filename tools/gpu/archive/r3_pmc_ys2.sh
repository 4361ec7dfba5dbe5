# fused YOLO stem: timing vs the unfused pair, then PMC passes (kernel-trace + counters only)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ys2; mkdir -p $OUT
timeout -k 10 120 python3 tools/stem2_probe.py > $OUT/times.txt 2>&1 || exit $?
cat $OUT/times.txt
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- \
    python3 tools/stem2_probe.py --only-fused --iters 2 > $OUT/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; head -5 $OUT/summary.txt
