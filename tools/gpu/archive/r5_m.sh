# Round 5 (m): v12 as a per-wave DMA ring (+ 32x64 / 64x32 / 64x64 tiles) -- kernel tests,
# graph-timed tile matrix at b1 / b8, edge A/B without / with the family
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5m}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "skinny or tile_count or canary or dual or every_tile" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest.txt
TL=90,94,101,103,108,109,110,111,112,113,114,115,116
for b in 1 8; do
  timeout -k 10 300 python -u tools/tile_probe.py --graph --batch $b --iters 20 --tiles $TL \
    --only s4.c2,s4.c2s,s3.c2,s3.c2s,s4.c1,s4.c3,s3.c1,s3.c3,s1.c3,s1.c1,s1.c2,s2.c3 > gpurun_out/${T}_tiles_b$b.md 2>&1 || { tail -20 gpurun_out/${T}_tiles_b$b.md; exit 1; }
done
cat gpurun_out/${T}_tiles_b1.md gpurun_out/${T}_tiles_b8.md
timeout -k 10 600 python -u tools/edge_ab.py --arms "KVEDGE_TILE_LIMIT=108;KVEDGE_TILE_LIMIT=0" --batches 1,8,64 --rounds 2 > gpurun_out/${T}_edge_ab.jsonl 2>gpurun_out/${T}_edge_ab.err || { tail -20 gpurun_out/${T}_edge_ab.err; exit 1; }
grep summary gpurun_out/${T}_edge_ab.jsonl
