# Round 6 (z8): YOLOv8n P3 Detect stem Cout split 128 + 16 (default) vs 80 + 64
# (KVEDGE_DIRECT_SPLIT=balanced), alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z8}
for r in 1 2; do
  for arm in greedy balanced; do
    if [ $arm = balanced ]; then export KVEDGE_DIRECT_SPLIT=balanced; else unset KVEDGE_DIRECT_SPLIT; fi
    KVEDGE_EDGE= timeout -k 10 600 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/${T}_${arm}_$r.txt 2>>gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
    echo "$arm $r: $(python tools/bench_line.py gpurun_out/${T}_${arm}_$r.txt)"
  done
done
