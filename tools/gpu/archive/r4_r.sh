# Round 4 (r): YOLO bench A/B on one box: NMS with the greedy prefetch (_C.so) vs without (_C_ab.so)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4r}
for r in 1 2; do
  for lib in _C.so _C_ab.so; do
    KVEDGE_LIB=$lib timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_${lib}_$r.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo_${lib}_$r.txt; exit 1; }
    echo "$lib $r $(grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo_${lib}_$r.txt | head -1)"
  done
done
