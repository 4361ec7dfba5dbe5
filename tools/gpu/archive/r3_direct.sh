# direct-conv changes (stride-2 column de-interleave, DMA/store wave roles): numerics, YOLO op roofline, bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $P tests/test_kernels_gpu.py -k "direct or canary" > gpurun_out/pytest_direct.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_direct.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/yolo_op_roofline_b192_v2.md 2> gpurun_out/yolo_op_roofline.err && \
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/bench_yolo.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/bench_resnet.log 2>&1
rc=$?
grep "^| 0 \|^| [1-9] \|^| 4[89] \|^| 5[0-9] \|Forward" gpurun_out/yolo_op_roofline_b192_v2.md
tail -n 1 gpurun_out/bench_yolo.log | cut -c1-200; tail -n 1 gpurun_out/bench_resnet.log | cut -c1-200
exit $rc
