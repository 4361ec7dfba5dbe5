# Round 5 (g): slices x streams sweep at the bench's 640-image slice (same box, alternating)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5g}
for i in 1 2; do
  for cfg in "1280 2" "1920 3" "2560 4" "1920 2"; do set -- $cfg
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" --yolo 0 --batch $1 --streams $2 > gpurun_out/${T}_b$1_s$2_$i.txt 2>&1 || { tail -20 gpurun_out/${T}_b$1_s$2_$i.txt; exit 1; }
    echo "b$1 s$2 run $i $(grep -o '"value": [0-9.]*' gpurun_out/${T}_b$1_s$2_$i.txt | head -1)"
  done
done
