set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_kernels_gpu.py > gpurun_out/pytest_kernels.log 2>&1 && \
timeout -k 10 300 python tools/tile_probe.py --batch 640 --iters 10 \
    --only s2.c1,s2.c3,s3.c1,s3.c3,s4.c3,s2.c2,s3.c2,s4.c2 --tiles 6,24,25,26,28,29,30,31 \
    > gpurun_out/tile_probe16.md 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov8n --steps 20 --warmup 3 > gpurun_out/bench_yolo.log 2>&1
rc=$?
for f in pytest_kernels bench bench_yolo; do echo "== $f"; tail -n 1 gpurun_out/$f.log | cut -c1-200; done
cat gpurun_out/tile_probe16.md
exit $rc
