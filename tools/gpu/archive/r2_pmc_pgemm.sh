# PMC passes on the s3/s4 expand+residual 1x1 layers: glds best tile vs the v5 persistent tile.
set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_layer.sh s3.c3 29 gpurun_out/pmc_s3c3_t29 && \
bash tools/pmc_layer.sh s3.c3 58 gpurun_out/pmc_s3c3_t58 && \
bash tools/pmc_layer.sh s3.c3 6 gpurun_out/pmc_s3c3_t6 && \
bash tools/pmc_layer.sh s3.c3 61 gpurun_out/pmc_s3c3_t61
rc=$?
for d in gpurun_out/pmc_s3c3_t*; do echo "== $d"; cat $d/summary.txt; done
exit $rc
