# Round 6 (k): full default bench (headline + edge + YOLOv8n) with the v14 tiles in the
# tuner's table (limit 0) vs without them (limit 117), alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6k}
for r in 1 2; do
for lim in 0 117; do
  KVEDGE_TILE_LIMIT=$lim timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_b_${lim}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "limit=$lim $(python tools/bench_line.py gpurun_out/${T}_b_${lim}_$r.txt)"
done
done
