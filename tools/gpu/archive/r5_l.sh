# Round 5 (l): the whole GPU tier with the v12 family + new tail gate; b64 tail-gate A/B; in-graph
# tables of the b1 / b8 edge steps
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5l}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.txt
timeout -k 10 400 python -u tools/edge_ab.py --arms "KVEDGE_TAIL1_MIN_ROWS=32768;KVEDGE_TAIL1_MIN_ROWS=1000000000" --batches 64 --rounds 2 > gpurun_out/${T}_tail64.jsonl 2>gpurun_out/${T}_tail64.err || { tail -20 gpurun_out/${T}_tail64.err; exit 1; }
grep summary gpurun_out/${T}_tail64.jsonl
run() {  # tag model batch streams
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_$1 -o gl \
    -- python3 tools/graph_layers.py run --model $2 --batch $3 --streams $4 --reps 20 --labels gpurun_out/${T}_$1_labels.json \
    > gpurun_out/${T}_$1.log 2>&1 || { tail -20 gpurun_out/${T}_$1.log; return 1; }
  python3 tools/graph_layers.py summarize gpurun_out/${T}_$1 --reps 20 --labels gpurun_out/${T}_$1_labels.json \
    > gpurun_out/${T}_$1.md 2>&1 || { tail -20 gpurun_out/${T}_$1.md; return 1; }
  head -4 gpurun_out/${T}_$1.md | tail -1
  rm -rf gpurun_out/${T}_$1
}
run rn_b1 resnet50 1 1 && run rn_b8 resnet50 8 1
