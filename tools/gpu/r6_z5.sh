# Round 6 (z5): bench-config parity tests with the cross-slice consistency checks
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z5}
timeout -k 10 600 python -u -m pytest tests/test_bench_config_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
