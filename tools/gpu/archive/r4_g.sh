# Round 4 (g): seam order (s3 deep residual ring first); PMC of the direct family and seams; bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4g}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "seam or tile_count" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
bash tools/gpu/r4_pmc_direct.sh > gpurun_out/${T}_pmc_direct.txt 2>&1 || { tail -20 gpurun_out/${T}_pmc_direct.txt; exit 1; }
cat gpurun_out/${T}_pmc_direct.txt
bash tools/gpu/r4_pmc_seam.sh > gpurun_out/${T}_pmc_seam.txt 2>&1 || { tail -20 gpurun_out/${T}_pmc_seam.txt; exit 1; }
cut -c1-400 gpurun_out/${T}_pmc_seam.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_resnet.txt 2>&1 || { tail -5 gpurun_out/${T}_resnet.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_resnet.txt | head -1
