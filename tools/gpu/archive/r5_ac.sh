# Round 5 (ac): every tile on ResNet-50's stage-3/4 layers at the edge batch 64 (graph-timed):
# where the K-serial stage-4 GEMMs (M = 3136, K up to 4608) stand against split-K / skinny
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ac}
timeout -k 10 600 python -u tools/tile_probe.py --batch 64 --graph --only s3.c1,s3.c2,s3.c3,s4.c1,s4.c2,s4.c3,s4.c2s,s3.c2s,s4.c1a --iters 20 > gpurun_out/${T}_tiles_b64.md 2>gpurun_out/${T}_tiles.err || { tail -20 gpurun_out/${T}_tiles.err; exit 1; }
echo done
