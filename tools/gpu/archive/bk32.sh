set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > gpurun_out/kern_tests.log 2>&1 && \
timeout -k 10 400 python tools/tile_probe.py --batch 640 --iters 10 --only s2.c2,s3.c2,s4.c2,s3.c1,s3.c3,s1.c2 --tiles 0,6,13,18,19,22,23,24 > gpurun_out/tile_probe_bk32.md 2>&1
rc=$?; tail -n 3 gpurun_out/kern_tests.log; cat gpurun_out/tile_probe_bk32.md; exit $rc
