set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/pmc_layer.sh s3.c3 6 gpurun_out/pmc_s3c3_t6 > gpurun_out/pmc_s3c3.log 2>&1 && \
bash tools/pmc_layer.sh s3.c3 22 gpurun_out/pmc_s3c3_t22 >> gpurun_out/pmc_s3c3.log 2>&1
rc=$?; cat gpurun_out/pmc_s3c3_t6/summary.txt gpurun_out/pmc_s3c3_t22/summary.txt | grep -v "at::\|rocclr"; exit $rc
