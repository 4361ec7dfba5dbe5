# Round 6 (m): headline, v14 with its persistent forms (limit 0) vs without them (119) vs no
# v14 at all (117), alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6m}
for r in 1 2; do
for lim in 0 119 117; do
  KVEDGE_TILE_LIMIT=$lim KVEDGE_BENCH_YOLO=0 KVEDGE_EDGE= timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 > gpurun_out/${T}_b_${lim}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "limit=$lim $(python tools/bench_line.py gpurun_out/${T}_b_${lim}_$r.txt)"
done
done
