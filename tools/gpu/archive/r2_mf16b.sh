set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_kernels_gpu.py tests/test_models_gpu.py > gpurun_out/pytest_kernels.log 2>&1 && \
timeout -k 10 300 python tools/tile_probe.py --batch 640 --iters 10 \
    --only s2.c1,s2.c3,s3.c1,s3.c3,s4.c3 --tiles 29,32,33,36,39,43,49,50,51 \
    > gpurun_out/tile_probe_stream16.md 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov8n --steps 20 --warmup 3 > gpurun_out/bench_yolo.log 2>&1 && \
bash tools/gpu_check.sh fwd fwdyolo > gpurun_out/prof_steps.log 2>&1
rc=$?
for f in pytest_kernels bench bench_yolo; do echo "== $f"; tail -n 1 gpurun_out/$f.log | cut -c1-200; done
cat gpurun_out/tile_probe_stream16.md; head -24 gpurun_out/fwd_summary.md
exit $rc
