# Round 6 (d): in-graph per-layer tables of the b1280 bench graph, KVEDGE_YSUB=1 vs 0
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6d}
for ys in 1 0; do
  d=gpurun_out/${T}_gl_$ys
  KVEDGE_YSUB=$ys timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
    python3 tools/graph_layers.py run --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
  python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
  rm -rf $d
  head -4 ${d}.md | tail -2
done
