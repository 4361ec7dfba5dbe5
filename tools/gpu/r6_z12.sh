# Round 6 (z12): PMC of the v14 tile on s3.c2 (b640) after keeping B0 in registers (KV_PP_KEEPB) --
# LDS-DMA staging (KVEDGE_PP_ABL 0 / 2 / 4): what the staging costs
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z12}
for A in 0; do
  OUT=gpurun_out/${T}_pmc_$A; mkdir -p $OUT
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
             "TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TD_BUSY_max TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    i=$((i+1))
    KVEDGE_PP_ABL=$A timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- \
      python3 tools/pp_abl.py --layer s3.c2 --batch 640 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  done
  echo "== abl $A"
  python3 tools/pmc_raw.py $OUT --match conv_pp_kernel
done
