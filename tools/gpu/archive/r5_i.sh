# Round 5 (i): v12 skinny edge-batch family -- kernel tests, same-box edge A/B without / with
# the family, in-graph table of the batch-1 step with it
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5i}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "skinny or tile_count or canary or dual or every_tile" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest.txt
timeout -k 10 600 python -u tools/edge_ab.py --arms 108,0 --batches 1,8,64 --rounds 2 > gpurun_out/${T}_edge_ab.jsonl 2>gpurun_out/${T}_edge_ab.err || { tail -20 gpurun_out/${T}_edge_ab.err; exit 1; }
grep summary gpurun_out/${T}_edge_ab.jsonl
run() {  # tag model batch streams
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_$1 -o gl \
    -- python3 tools/graph_layers.py run --model $2 --batch $3 --streams $4 --reps 20 --labels gpurun_out/${T}_$1_labels.json \
    > gpurun_out/${T}_$1.log 2>&1 || { tail -20 gpurun_out/${T}_$1.log; return 1; }
  python3 tools/graph_layers.py summarize gpurun_out/${T}_$1 --reps 20 --labels gpurun_out/${T}_$1_labels.json \
    > gpurun_out/${T}_$1.md 2>&1 || { tail -20 gpurun_out/${T}_$1.md; return 1; }
  head -4 gpurun_out/${T}_$1.md | tail -1
  rm -rf gpurun_out/${T}_$1
}
run rn_b1 resnet50 1 1
