# YOLOv8n A/B: autotuner without (KVEDGE_TILE_LIMIT=58) and with the v6 family, 3 pairs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python tools/tune_report.py --model yolov8n > gpurun_out/tune_yolo.txt 2>&1 || exit $?
for i in 1 2 3; do
for lim in 58 0; do
KVEDGE_TILE_LIMIT=$lim timeout -k 10 150 python bench.py --model yolov8n --steps 30 --warmup 5 2>/dev/null | grep metric | sed "s/^/{\"tile_limit\": $lim, \"r\": /; s/$/}/" >> gpurun_out/ab_yolo_nloop.jsonl || exit $?
done; done
