# Round 5 (ai): in-graph refine with a wider runner-up net (tiles within 60 % of the isolated
# best, up to 4 per layer) vs the default (25 %, 2) at the edge batches, same 60 s budget
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ai}
timeout -k 10 1000 python -u tools/edge_ab.py --arms "KVEDGE_GRAPH_REFINE_S=60;KVEDGE_GRAPH_REFINE_S=60,KVEDGE_ALT_TOL=0.6,KVEDGE_ALT_MAX=4" --batches 64,8 --rounds 2 > gpurun_out/${T}_edge.jsonl 2>gpurun_out/${T}_edge.err || { tail -20 gpurun_out/${T}_edge.err; exit 1; }
grep summary gpurun_out/${T}_edge.jsonl
