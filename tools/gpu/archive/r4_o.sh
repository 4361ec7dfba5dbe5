# Round 4 (o): seam XP forms (cross-step fragment prefetch) numerics + same-box probe;
# then the r4_n set (tail-ring A/B, edge profiles)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4o}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "seam or tail or tile_count" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u tools/seam_probe.py --batch 640 > gpurun_out/${T}_seam_probe.md 2> gpurun_out/${T}_probe.err || { tail -5 gpurun_out/${T}_probe.err; exit 1; }
cut -c1-900 gpurun_out/${T}_seam_probe.md
TAG=r4n bash tools/gpu/r4_n.sh
