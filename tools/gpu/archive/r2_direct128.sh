# Direct 3x3 (opaque LDS DMA): numerics, then direct vs glds tiles on the stage-1/2 conv2.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "direct or every_tile or canary" > gpurun_out/pytest_direct128.log 2>&1 && \
timeout -k 10 300 python tools/tile_probe.py --batch 640 --iters 10 --tiles 6,29,54,55,56,57 --only s1.c2,s2.c2 > gpurun_out/probe_direct128.md 2>&1
rc=$?
tail -n 3 gpurun_out/pytest_direct128.log
grep -v amdgpu.ids gpurun_out/probe_direct128.md
exit $rc
