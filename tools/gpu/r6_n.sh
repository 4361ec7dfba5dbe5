# Round 6 (n): in-graph layer tables of ResNet-50 at b640 on ONE stream vs b1280 on two (the
# bench), same box: where does the second slice help, where does it interfere
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6n}
for spec in "640 1" "1280 2"; do
  set -- $spec
  d=gpurun_out/${T}_gl_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
    python3 tools/graph_layers.py run --batch $1 --streams $2 --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
  python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
  rm -rf $d
  echo "b$1 s$2 $(head -4 ${d}.md | tail -1)"
done
