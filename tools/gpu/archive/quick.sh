# Kernel tests (subset via $KSEL), full GPU tests, both benches, forward profiles.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov8n --steps 20 --warmup 3 > gpurun_out/bench_yolo.log 2>&1 && \
bash tools/gpu_check.sh ${PROF:-fwd fwdyolo} > gpurun_out/prof_steps.log 2>&1
rc=$?
for f in pytest_gpu bench bench_yolo; do echo "== $f"; tail -n 2 gpurun_out/$f.log; done
exit $rc
