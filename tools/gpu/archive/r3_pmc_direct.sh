# PMC passes over the YOLO Detect P3 direct 3x3 (64 -> 128 @80x80, b192) and the stem kernels
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_direct; mkdir -p $OUT
timeout -k 10 120 python3 tools/conv_probe.py --shape 192,80,80,64,128,3,1 --tiles 54,55,56,57 > $OUT/times.txt 2>&1 || exit $?
cat $OUT/times.txt
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- \
    python3 tools/conv_probe.py --shape 192,80,80,64,128,3,1 --tiles 55 --iters 3 > $OUT/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; head -6 $OUT/summary.txt
bash tools/gpu/r3_pmc_stem.sh
