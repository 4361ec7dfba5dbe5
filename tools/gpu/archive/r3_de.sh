# direct-epilogue tiles: numerics, probes (single + concurrent), then bench + b640 roofline + edge profiles
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $P tests/test_kernels_gpu.py -k "every_tile and (80 or 81 or 82 or 83) or dual_fused and (80 or 81 or 82 or 83) or test_tile_count or even_pixels or tail_fused" > gpurun_out/pytest_de.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_de.log
[ $rc -ne 0 ] && exit $rc
L=s3.c2,s4.c2,s2.c2,s3.c1,s4.c1,s4.c3,s3.c3,s3.c1a,s4.c1a,s2.c2s,s3.c2s,s4.c2s,s2.c1
T=29,30,70,75,80,81,82,83
timeout -k 10 600 python -u tools/tile_probe.py --batch 640 --iters 10 --tiles $T --only $L > gpurun_out/de_probe.md 2>&1 && cat gpurun_out/de_probe.md && \
timeout -k 10 600 python -u tools/tile_probe.py --batch 640 --iters 10 --concurrent 2 --tiles $T --only $L > gpurun_out/de_probe_c2.md 2>&1 && cat gpurun_out/de_probe_c2.md && \
timeout -k 10 300 python -u tools/dual_probe.py --batch 640 --tiles 30,70,75,80,81,82 > gpurun_out/de_dual.md 2>&1 && cat gpurun_out/de_dual.md && \
bash tools/gpu/r3_bench_prof.sh
