# Round 5 (z): edge serving re-check of two stream slices at b8 / b64 (round 3 measured them slower)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5z}
timeout -k 10 600 python -u tools/edge_ab.py --arms "KVEDGE_EDGE_STREAMS=1;KVEDGE_EDGE_STREAMS=2" --batches 8,64 --rounds 2 > gpurun_out/${T}_streams.jsonl 2>gpurun_out/${T}_streams.err || { tail -20 gpurun_out/${T}_streams.err; exit 1; }
grep summary gpurun_out/${T}_streams.jsonl
