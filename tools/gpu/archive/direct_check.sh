set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "direct or stem or every_tile or canary or tile_count" > gpurun_out/direct_test.log 2>&1 && \
timeout -k 10 120 python tools/stem_probe.py > gpurun_out/stem_new.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model yolov8n --steps 20 --warmup 3 > gpurun_out/bench_yolo.log 2>&1
rc=$?
for f in direct_test stem_new pytest_gpu bench bench_yolo; do echo "== $f"; tail -n 3 gpurun_out/$f.log; done
exit $rc
