# Round 5 (q): in-graph tables of the ResNet-50 b1280 bench step and the b64 edge step (final tree)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5p}
run() {  # tag model batch streams
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_$1 -o gl \
    -- python3 tools/graph_layers.py run --model $2 --batch $3 --streams $4 --reps 20 --labels gpurun_out/${T}_$1_labels.json \
    > gpurun_out/${T}_$1.log 2>&1 || { tail -20 gpurun_out/${T}_$1.log; return 1; }
  python3 tools/graph_layers.py summarize gpurun_out/${T}_$1 --reps 20 --labels gpurun_out/${T}_$1_labels.json \
    > gpurun_out/${T}_$1.md 2>&1 || { tail -20 gpurun_out/${T}_$1.md; return 1; }
  head -4 gpurun_out/${T}_$1.md | tail -1
  rm -rf gpurun_out/${T}_$1
}
run rn_b1280 resnet50 1280 2 && run rn_b64 resnet50 64 1
