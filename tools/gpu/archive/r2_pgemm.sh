# v5 persistent GEMM: kernel tests first (fault -> stop), then the tile probe on the mid-network layers.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $P tests/test_kernels_gpu.py -k "pgemm or every_tile or dual_fused or canary or tile_count" > gpurun_out/pytest_pgemm.log 2>&1 && \
timeout -k 10 500 python tools/tile_probe.py --batch 640 --iters 10 --tiles ${TILES:-6,24,25,27,28,29,30,58,59,60,61,62,63,64,65} --only ${ONLY:-s2.c2,s3.c2,s4.c2,s3.c1,s3.c3,s4.c3,s4.c1,s3.c1a,s4.c1a} > gpurun_out/tile_probe_pgemm.md 2>&1
rc=$?
tail -n 3 gpurun_out/pytest_pgemm.log
cat gpurun_out/tile_probe_pgemm.md 2>/dev/null | grep -v amdgpu.ids
exit $rc
