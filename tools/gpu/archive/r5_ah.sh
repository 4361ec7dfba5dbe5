# Round 5 (ah): PMC passes over the ResNet-50 dual 1x1s (conv3 + strided downsample as one
# GEMM) on their graph tile (xp/bk32/de:80) at b640: where the 0.3-0.4-of-floor time goes
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ah}
for L in s2.dual s3.dual; do
  OUT=gpurun_out/${T}_$L; mkdir -p $OUT; i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- \
      python3 tools/dual_probe.py --only $L --tiles 80 --iters 3 --batch 640 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1 || true
  echo "== $L"; grep -E "kernel|conv_glds" $OUT/summary.txt | cut -c1-400
done
