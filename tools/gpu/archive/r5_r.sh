# Round 5 (r): fused C2f diagnostics (which phase holds the time) + correctness with y staging
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5r}
timeout -k 10 300 python -u tools/c2f_probe.py --batch 256 --strips 40 --diags 0,1,2,4,6,7,8,9,10 > gpurun_out/${T}_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_probe.txt; exit 1; }
cat gpurun_out/${T}_probe.txt
KVEDGE_C2F_DIAG=8 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "c2f16" > gpurun_out/${T}_pytest8.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest8.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest8.txt
