set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 bash tools/pmc_layer.sh s3.c2 30 gpurun_out/pmc30 && \
timeout -k 10 400 bash tools/pmc_layer.sh s3.c2 68 gpurun_out/pmc68 && \
cat gpurun_out/pmc30/summary.txt gpurun_out/pmc68/summary.txt
