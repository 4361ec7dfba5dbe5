# Round 4 (c): seam forms with A in VGPRs; numerics + probe + bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4c}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "seam or every_tile or canary" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u tools/seam_probe.py --batch 640 > gpurun_out/${T}_seam_probe.md 2>&1 || { cat gpurun_out/${T}_seam_probe.md; exit 1; }
cat gpurun_out/${T}_seam_probe.md
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench.txt 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/${T}_bench.txt | head -1
