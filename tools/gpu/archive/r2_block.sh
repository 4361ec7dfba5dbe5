# Fused layer-1 bottleneck body: numerics first (fault -> stop), then fused vs unfused timing.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_block_gpu.py > gpurun_out/pytest_block.log 2>&1 && \
timeout -k 10 300 python tools/block_probe.py --batch 640 > gpurun_out/block_probe.md 2>&1
rc=$?
tail -n 5 gpurun_out/pytest_block.log
grep -v amdgpu.ids gpurun_out/block_probe.md
exit $rc
