# Round 6 (z9): NMS fallback sorts only the keys below the top set -- NMS / YOLO tests, probe
# at b192 / b256, YOLOv8n bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z9}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "nms or yolo" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for b in 192 256; do
timeout -k 10 300 python -u tools/nms_probe.py --batch $b > gpurun_out/${T}_nms$b.txt 2>&1 || { tail -20 gpurun_out/${T}_nms$b.txt; exit 1; }
grep -E "max over|diag 0" gpurun_out/${T}_nms$b.txt
done
KVEDGE_EDGE= timeout -k 10 600 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/${T}_yolo.txt 2>gpurun_out/${T}_yolo.err || { tail -20 gpurun_out/${T}_yolo.err; exit 1; }
python tools/bench_line.py gpurun_out/${T}_yolo.txt
