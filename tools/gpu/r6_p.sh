# Round 6 (p): NMS top set rank-sorted (kSel 768) -- GPU tests touching NMS / YOLO, the NMS probe
# at the bench's slice size, and the bench's YOLOv8n number
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6p}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "nms or yolo" --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 300 python -u tools/nms_probe.py --batch 256 > gpurun_out/${T}_nms.txt 2>&1 || { tail -20 gpurun_out/${T}_nms.txt; exit 1; }
cat gpurun_out/${T}_nms.txt
KVEDGE_EDGE= timeout -k 10 600 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/${T}_yolo.txt 2>gpurun_out/${T}_yolo.err || { tail -20 gpurun_out/${T}_yolo.err; exit 1; }
tail -1 gpurun_out/${T}_yolo.txt
