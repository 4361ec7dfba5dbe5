# Round 4 (q): NMS rank sort + phase stamps; NMS / YOLO tests; YOLO bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4q}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bench_config_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread \
  -k "nms or yolo" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u tools/nms_probe.py --batch 192 > gpurun_out/${T}_nms.txt 2>&1 || { tail -5 gpurun_out/${T}_nms.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_nms.txt
timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo.txt | head -1
