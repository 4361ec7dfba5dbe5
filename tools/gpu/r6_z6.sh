# Round 6 (z6): edge batches with the v9 seams allowed at stage 3 (SEAM_MIN_WGS 64 / 32) vs the
# default gate (256), alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z6}
timeout -k 10 900 python -u tools/edge_ab.py --arms "KVEDGE_SEAM_MIN_WGS=256;KVEDGE_SEAM_MIN_WGS=64;KVEDGE_SEAM_MIN_WGS=32" --batches 32,64 --rounds 2 > gpurun_out/${T}_seam_edge.jsonl 2>&1 || { tail -20 gpurun_out/${T}_seam_edge.jsonl; exit 1; }
grep summary gpurun_out/${T}_seam_edge.jsonl
