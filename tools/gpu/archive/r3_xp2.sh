# XP tiles after the BK32/MF16 swizzle fix: numerics, probe at b640, PMC at b640, bench.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $P tests/test_kernels_gpu.py -k "every_tile and (68 or 69 or 70 or 71 or 72 or 73) or dual_fused and (68 or 69 or 70 or 71 or 72 or 73) or canary or test_tile_count" > gpurun_out/pytest_xp.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_xp.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/tile_probe.py --batch 640 --iters 10 --tiles 24,29,30,31,68,69,70,71,72,73 --only s3.c2,s4.c2,s2.c2,s3.c1,s4.c1,s4.c3,s3.c1a,s4.c1a,s2.c2s,s3.c2s,s4.c2s > gpurun_out/xp_probe.md 2>&1 && cat gpurun_out/xp_probe.md && \
PMC_BATCH=640 timeout -k 10 400 bash tools/pmc_layer.sh s3.c2 30 gpurun_out/pmc30 && \
PMC_BATCH=640 timeout -k 10 400 bash tools/pmc_layer.sh s3.c2 68 gpurun_out/pmc68 && \
cat gpurun_out/pmc30/summary.txt gpurun_out/pmc68/summary.txt | grep conv_glds && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?
tail -n 1 gpurun_out/bench.log | cut -c1-400
exit $rc
