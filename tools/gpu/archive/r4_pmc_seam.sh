# PMC of the s3 seam (16-KB stages, tile 7) and the s2 seam (4-wave, tile 0), one pass per
# counter group (counters only with --kernel-trace; never with trace domains)
set -o pipefail
mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
for sh in "s3 7" "s2 0"; do set -- $sh  # kSmTiles indices: s3 first form, s2 first form
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/$1_a -o a \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA \
    -- python3 tools/seam_one.py --shape $1 --tile $2 > gpurun_out/pmc/$1_a.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/$1_b -o b \
    --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE \
    -- python3 tools/seam_one.py --shape $1 --tile $2 > gpurun_out/pmc/$1_b.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/$1_c -o c \
    --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
    -- python3 tools/seam_one.py --shape $1 --tile $2 > gpurun_out/pmc/$1_c.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/pmc "s3_*/*_counter_collection.csv" > gpurun_out/pmc/summary_s3.md 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc "s2_*/*_counter_collection.csv" > gpurun_out/pmc/summary_s2.md 2>&1
cat gpurun_out/pmc/summary_s3.md gpurun_out/pmc/summary_s2.md
