# Round 5 (b): in-graph tile refinement A/B on one box (KVEDGE_GRAPH_REFINE=0 vs default),
# then the in-graph per-layer table of the refined bench graph.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5b}
for i in 1 2; do
  KVEDGE_GRAPH_REFINE=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" --yolo 0 > gpurun_out/${T}_off$i.txt 2>&1 || { tail -20 gpurun_out/${T}_off$i.txt; exit 1; }
  echo "off $i $(grep -o '"value": [0-9.]*' gpurun_out/${T}_off$i.txt | head -1)"
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" --yolo 0 > gpurun_out/${T}_on$i.txt 2>&1 || { tail -20 gpurun_out/${T}_on$i.txt; exit 1; }
  echo "on $i $(grep -o '"value": [0-9.]*' gpurun_out/${T}_on$i.txt | head -1) $(grep -o '"graph_refine": {[^}]*}' gpurun_out/${T}_on$i.txt)"
done
KVEDGE_GRAPH_REFINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_gl0 -o gl \
  -- python3 tools/graph_layers.py run --streams 2 --labels gpurun_out/${T}_gl0_labels.json \
  > gpurun_out/${T}_gl0.log 2>&1 || { tail -20 gpurun_out/${T}_gl0.log; exit 1; }
python3 tools/graph_layers.py summarize gpurun_out/${T}_gl0 --labels gpurun_out/${T}_gl0_labels.json \
  > gpurun_out/${T}_graph_layers_s2_norefine.md 2>&1 || { tail -20 gpurun_out/${T}_graph_layers_s2_norefine.md; exit 1; }
head -4 gpurun_out/${T}_graph_layers_s2_norefine.md | tail -1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_gl2 -o gl \
  -- python3 tools/graph_layers.py run --streams 2 --labels gpurun_out/${T}_gl2_labels.json \
  > gpurun_out/${T}_gl2.log 2>&1 || { tail -20 gpurun_out/${T}_gl2.log; exit 1; }
python3 tools/graph_layers.py summarize gpurun_out/${T}_gl2 --labels gpurun_out/${T}_gl2_labels.json \
  > gpurun_out/${T}_graph_layers_s2.md 2>&1 || { tail -20 gpurun_out/${T}_graph_layers_s2.md; exit 1; }
head -4 gpurun_out/${T}_graph_layers_s2.md | tail -1
