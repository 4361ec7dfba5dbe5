set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $P tests/test_kernels_gpu.py -k "every_tile and (74 or 75 or 76 or 77 or 78 or 79) or dual_fused and (74 or 75 or 76 or 77 or 78 or 79) or test_tile_count" > gpurun_out/pytest_bk32.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_bk32.log
[ $rc -ne 0 ] && exit $rc
L=s3.c2,s4.c2,s2.c2,s3.c1,s4.c1,s4.c3,s3.c3,s3.c1a,s4.c1a,s2.c2s,s3.c2s,s4.c2s,s2.c1,s2.c3
T=24,29,30,31,48,70,74,75,76,77,78,79
timeout -k 10 600 python -u tools/tile_probe.py --batch 640 --iters 10 --tiles $T --only $L > gpurun_out/bk32_probe.md 2>&1 && cat gpurun_out/bk32_probe.md && \
timeout -k 10 600 python -u tools/tile_probe.py --batch 640 --iters 10 --concurrent 2 --tiles $T --only $L > gpurun_out/bk32_probe_c2.md 2>&1 && cat gpurun_out/bk32_probe_c2.md && \
timeout -k 10 300 python -u tools/dual_probe.py --batch 640 --tiles 24,30,70,74,75,76,77,78,79 > gpurun_out/bk32_dual.md 2>&1 && cat gpurun_out/bk32_dual.md
