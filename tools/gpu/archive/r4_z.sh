# Round 4 (z): SPPF on packed int16 keys: numerics, per-op time (b192 slice), YOLO bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4z}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "sppf or upsample or yolo" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/${T}_yolo_op_roofline_b192.md 2> gpurun_out/${T}_yolo.err || { tail -5 gpurun_out/${T}_yolo.err; exit 1; }
grep -n "sppf\|Forward" gpurun_out/${T}_yolo_op_roofline_b192.md
timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo.txt | head -1
