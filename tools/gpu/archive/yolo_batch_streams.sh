# YOLOv8n two-stream bench at several per-GPU batches
set -o pipefail
mkdir -p gpurun_out
for b in 384 512 640 768 384; do
  timeout -k 10 200 python bench.py --model yolov8n --steps 20 --warmup 3 --batch $b 2>/dev/null | grep metric >> gpurun_out/yolo_batch_streams.jsonl || exit $?
done
