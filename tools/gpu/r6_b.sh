# Round 6 (b): in-graph tile A/B of the stage-2 entry 3x3/2 (and the s3/s4 ones) in the
# b1280 bench graph, candidates from the isolated tile probe
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6b}
timeout -k 10 600 python -u tools/layer_swap.py --match "3, 3, 2, 1" --tiles 29,74,75,76,80,82 > gpurun_out/${T}_swap.jsonl 2>gpurun_out/${T}_swap.err || { tail -20 gpurun_out/${T}_swap.err; exit 1; }
grep trial gpurun_out/${T}_swap.jsonl
