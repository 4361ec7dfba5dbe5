# PMC passes over the direct family (v10 direct-epilogue tile 105, asm fragment ring): the
# YOLO Detect P3 stem slice 64 -> 128 @80x80 (b192) and ResNet-50 stage-1 3x3 (b640)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_direct; mkdir -p $OUT
for sp in "p3 192,80,80,64,128,3,1 silu" "r1 640,56,56,64,64,3,1 relu"; do set -- $sp
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/$1_p$i -o p$i -- \
      python3 tools/conv_probe.py --shape $2 --act $3 --tiles 105 --iters 3 > $OUT/$1_p$i.log 2>&1 || exit $?
  done
  python3 tools/pmc_summary.py $OUT "$1_p*/*_counter_collection.csv" > $OUT/summary_$1.md 2>&1
  cut -c1-400 $OUT/summary_$1.md
done
