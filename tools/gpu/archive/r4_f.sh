# Round 4 (f): direct family with the asm LDS fragment ring; numerics + YOLO A/B + ResNet
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4f}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "direct or canary or seam or tile_count or splitk or every_tile or pair or nms" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_de.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo_de.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo_de.txt | head -1
KVEDGE_TILE_LIMIT=105 timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_base.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo_base.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo_base.txt | head -1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_resnet.txt 2>&1 || { tail -5 gpurun_out/${T}_resnet.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_resnet.txt | head -1
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/${T}_yolo_op_roofline_b192.md 2> gpurun_out/${T}_yolo.err || { tail -5 gpurun_out/${T}_yolo.err; exit 1; }
tail -n 4 gpurun_out/${T}_yolo_op_roofline_b192.md
timeout -k 10 400 python -u tools/op_roofline.py --model resnet50 --batch 640 --streams 2 > gpurun_out/${T}_resnet_op_roofline_b640.md 2> gpurun_out/${T}_resnet.err || { tail -5 gpurun_out/${T}_resnet.err; exit 1; }
tail -n 4 gpurun_out/${T}_resnet_op_roofline_b640.md
