set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
KVEDGE_STEM_THREADS=256 timeout -k 10 120 python tools/stem_probe.py > gpurun_out/stem256.log 2>&1 && \
KVEDGE_STEM_THREADS=512 timeout -k 10 120 python tools/stem_probe.py > gpurun_out/stem512.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k stem > gpurun_out/stem_test.log 2>&1 && \
KVEDGE_CHECKS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/checks_gpu.log 2>&1
rc=$?
tail -2 gpurun_out/stem256.log gpurun_out/stem512.log gpurun_out/stem_test.log gpurun_out/checks_gpu.log
exit $rc
