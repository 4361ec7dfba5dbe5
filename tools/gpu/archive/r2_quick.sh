# Kernel/model tests + both benches + forward profiles (fast iteration loop).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_kernels_gpu.py tests/test_models_gpu.py > gpurun_out/pytest_kernels.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov8n --steps 20 --warmup 3 > gpurun_out/bench_yolo.log 2>&1 && \
bash tools/gpu_check.sh ${PROF:-fwd fwdyolo} > gpurun_out/prof_steps.log 2>&1
rc=$?
for f in pytest_kernels bench bench_yolo; do echo "== $f"; tail -n 1 gpurun_out/$f.log | cut -c1-200; done
head -12 gpurun_out/fwd_yolo_summary.md
exit $rc
