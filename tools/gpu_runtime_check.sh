set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_runtime_gpu.py > gpurun_out/rt_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --native-loop --profile gpurun_out/profile_r50.json > gpurun_out/bench_native.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov8n --steps 10 --warmup 3 --profile gpurun_out/profile_yolo.json > gpurun_out/bench_yolo_prof.log 2>&1
rc=$?
tail -5 gpurun_out/rt_gpu.log; tail -3 gpurun_out/bench_native.log; tail -3 gpurun_out/bench_yolo_prof.log
exit $rc
