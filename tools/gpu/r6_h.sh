# Round 6 (h): headline with the v14 tile in the tuner's table (default) vs without it
# (KVEDGE_TILE_LIMIT=117), alternated on one box; then the in-graph layer table
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6h}
for r in 1 2; do
for lim in 0 117; do
  KVEDGE_TILE_LIMIT=$lim KVEDGE_BENCH_YOLO=0 KVEDGE_EDGE= timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 > gpurun_out/${T}_b_${lim}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "limit=$lim $(python tools/bench_line.py gpurun_out/${T}_b_${lim}_$r.txt)"
done
done
d=gpurun_out/${T}_gl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
  python3 tools/graph_layers.py run --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
rm -rf $d
head -4 ${d}.md | tail -2
