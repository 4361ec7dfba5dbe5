set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/pmc_layer.sh s3.c2 6 gpurun_out/pmc_s3c2_t6 > gpurun_out/pmc_s3c2.log 2>&1
rc=$?; grep -v "at::\|rocclr" gpurun_out/pmc_s3c2_t6/summary.txt; exit $rc
