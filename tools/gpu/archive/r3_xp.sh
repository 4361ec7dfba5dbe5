# v7 (XP) tiles: numerics on every case, then tile probe vs the v2 references at b640.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $P tests/test_kernels_gpu.py -k "every_tile and (68 or 69 or 70 or 71 or 72 or 73) or dual_fused and (68 or 69 or 70 or 71 or 72 or 73) or test_tile_count" > gpurun_out/pytest_xp.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_xp.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python -u tools/tile_probe.py --batch 640 --iters 10 --tiles 24,25,29,30,31,68,69,70,71,72,73 --only s3.c2,s4.c2,s2.c2,s3.c1,s4.c1,s4.c3,s3.c1a,s4.c1a,s2.c2s,s3.c2s,s4.c2s,s3.c3 > gpurun_out/xp_probe.md 2>&1 && \
timeout -k 10 300 python -u tools/dual_probe.py --batch 640 --tiles 24,30,68,69,70,71 > gpurun_out/xp_dual.md 2>&1
rc2=$?
cat gpurun_out/xp_probe.md gpurun_out/xp_dual.md
exit $rc2
