# Round 6 (a): baseline on this box -- default bench, per-tile times of the 3x3 / 1x1 GEMM
# layers at b640, the hipBLASLt yard-stick on the same box, PMC of tile 80 on s3.c2
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6a}
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.txt 2>gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python tools/bench_line.py gpurun_out/${T}_bench.txt
timeout -k 10 300 python -u tools/blas_ceiling.py --batch 640 > gpurun_out/${T}_blas.md 2>&1 || { tail -20 gpurun_out/${T}_blas.md; exit 1; }
cat gpurun_out/${T}_blas.md
timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --only s2.c2,s3.c2,s4.c2,s2.c2s,s3.c2s,s4.c2s,s3.c1,s4.c1,s3.c3-nores,s4.c3 --tiles 75,76,79,80,81,82,83 > gpurun_out/${T}_tiles.md 2>&1 || { tail -20 gpurun_out/${T}_tiles.md; exit 1; }
cat gpurun_out/${T}_tiles.md
PMC_BATCH=640 timeout -k 10 400 bash tools/pmc_layer.sh s3.c2 80 gpurun_out/${T}_pmc_s3c2 || exit 1
cat gpurun_out/${T}_pmc_s3c2/summary.txt
