# Round-2 GPU session: new + tightened GPU tests, big-batch benches, amd-smi format probe.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
(amd-smi metric -g 0 -u -m --json > gpurun_out/amdsmi_metric.json 2>&1 || true)
timeout -k 10 600 $P tests/test_chunking_gpu.py tests/test_bench_config_gpu.py \
    tests/test_models_gpu.py tests/test_runtime_gpu.py > gpurun_out/pytest_r2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 2048 --no-autotune \
    > gpurun_out/bench_b2048.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov8n --steps 10 --warmup 3 --batch 768 --no-autotune \
    > gpurun_out/bench_yolo_b768.log 2>&1
rc=$?
for f in pytest_r2 bench_b2048 bench_yolo_b768; do echo "== $f"; tail -n 3 gpurun_out/$f.log; done
exit $rc
