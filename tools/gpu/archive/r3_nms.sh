# NMS top-set + autotune host-hold: numerics, YOLO bench, ResNet bench with edge block, b1 profile
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_kernels_gpu.py -k "nms or splitk" tests/test_models_gpu.py tests/test_bench_config_gpu.py > gpurun_out/pytest_nms.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_nms.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/bench_yolo.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwd1 -o fwd1 -- python3 tools/profile_forward.py --batch 1 --reps 20 > gpurun_out/fwd1.log 2>&1 && \
python tools/profile_forward.py --summarize gpurun_out/fwd1/fwd1_kernel_trace.csv --reps 20 > gpurun_out/fwd_b1.md
rc=$?
tail -n 1 gpurun_out/bench_yolo.log | cut -c1-200; tail -n 1 gpurun_out/bench.log | cut -c1-200; grep -o '"edge": \[[^]]*\]' gpurun_out/bench.log
head -12 gpurun_out/fwd_b1.md
exit $rc
