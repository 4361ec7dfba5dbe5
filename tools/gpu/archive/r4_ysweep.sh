# Round 4: YOLOv8n bench batch re-check on the final tree, one box, alternating order
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4ys}
for b in 384 512 256 384 512 256; do
  timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" --batch $b > gpurun_out/${T}_b$b.txt 2>&1 || { tail -5 gpurun_out/${T}_b$b.txt; exit 1; }
  echo "batch $b: $(grep -o '"value": [0-9.]*' gpurun_out/${T}_b$b.txt | head -1)" | tee -a gpurun_out/${T}_sweep.txt
done
