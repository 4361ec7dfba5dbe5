# weights settled out of the wait-count pass (stem12, yolo_stem2): numerics, probes, benches
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_models_gpu.py tests/test_kernels_gpu.py -k "stem or yolo or nms or avgpool" > gpurun_out/pytest_settle.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_settle.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/stem2_probe.py > gpurun_out/stem2_times.txt 2>&1 && cat gpurun_out/stem2_times.txt && \
timeout -k 10 120 python3 tools/stem_probe.py --batch 640 > gpurun_out/stem_times.txt 2>&1 && tail -n 4 gpurun_out/stem_times.txt && \
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/bench_yolo.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?
tail -n 1 gpurun_out/bench_yolo.log | cut -c1-200; tail -n 1 gpurun_out/bench.log | cut -c1-200; grep -o '"edge": \[[^]]*\]' gpurun_out/bench.log
exit $rc
