# Round 5 (j): v12 tile matrix at batch 1 / 8 for the stage-3/4 layers; stage-1 tail gate A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5j}
TL=86,90,94,101,103,108,109,110,111,112,113,114,115,116
for b in 1 8; do
  timeout -k 10 300 python -u tools/tile_probe.py --batch $b --iters 50 --tiles $TL \
    --only s4.c2,s4.c2s,s3.c2,s3.c2s,s4.c1,s4.c3,s3.c1,s3.c3,s1.c3,s1.c1,s1.c2,s2.c3 > gpurun_out/${T}_tiles_b$b.md 2>&1 || { tail -20 gpurun_out/${T}_tiles_b$b.md; exit 1; }
done
cat gpurun_out/${T}_tiles_b1.md
timeout -k 10 600 python -u tools/edge_ab.py --arms "KVEDGE_TAIL1_MIN_ROWS=0;KVEDGE_TAIL1_MIN_ROWS=4096;KVEDGE_TAIL1_MIN_ROWS=32768" --batches 1,8 --rounds 2 > gpurun_out/${T}_tail_ab.jsonl 2>gpurun_out/${T}_tail_ab.err || { tail -20 gpurun_out/${T}_tail_ab.err; exit 1; }
grep summary gpurun_out/${T}_tail_ab.jsonl
