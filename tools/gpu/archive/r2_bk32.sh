# BK = 32 deep-ring 256x256 8-wave tiles: every-tile numerics, then the stage-3/4 convs.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "every_tile or tile_count or dual_fused or canary" > gpurun_out/pytest_bk32.log 2>&1 && \
timeout -k 10 400 python tools/tile_probe.py --batch 640 --iters 10 --tiles 25,30,32,33,34 --only s3.c2,s4.c2,s3.c1,s4.c1,s3.c1a,s4.c1a,s2.c2 > gpurun_out/probe_bk32.md 2>&1
rc=$?
tail -n 3 gpurun_out/pytest_bk32.log
grep -v amdgpu.ids gpurun_out/probe_bk32.md
exit $rc
