# Round 5 (a): baseline on this box -- bench, then the in-graph per-layer table of the bench
# graph (tools/graph_layers.py) for two slices (the bench) and one.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5a}
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench.txt 2>&1 || { tail -20 gpurun_out/${T}_bench.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_bench.txt | head -1
for S in 2 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_gl$S -o gl \
    -- python3 tools/graph_layers.py run --streams $S --labels gpurun_out/${T}_gl${S}_labels.json \
    > gpurun_out/${T}_gl${S}.log 2>&1 || { tail -20 gpurun_out/${T}_gl${S}.log; exit 1; }
  python3 tools/graph_layers.py summarize gpurun_out/${T}_gl$S --labels gpurun_out/${T}_gl${S}_labels.json \
    > gpurun_out/${T}_graph_layers_s$S.md 2>&1 || { tail -20 gpurun_out/${T}_graph_layers_s$S.md; exit 1; }
  head -4 gpurun_out/${T}_graph_layers_s$S.md | tail -1
done
