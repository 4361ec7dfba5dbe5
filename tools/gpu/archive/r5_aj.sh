# Round 5 (aj): deeper-ring direct-epilogue tiles for the short-K GEMMs (xp tiles 18-20 = conv
# tiles 86-88: 256x128 / 128x256 D=3 BK=64, 256x256 D=5 BK=32) -- dual probe on them, every-tile
# test on the new indices, then the full bench alternated with the library without them
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5aj}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "tile_count or every_tile or dual or canary" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 300 python -u tools/dual_probe.py --batch 640 --tiles 80,81,86,87,88 > gpurun_out/${T}_dual.md 2>gpurun_out/${T}_dual.err || { tail -20 gpurun_out/${T}_dual.err; exit 1; }
cat gpurun_out/${T}_dual.md
timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --concurrent 2 --only s2.c1,s3.c1,s3.c3,s4.c1,s4.c3,s2.c3 --tiles 75,76,80,81,83,86,87,88 --iters 10 > gpurun_out/${T}_tiles.md 2>gpurun_out/${T}_tiles.err || { tail -20 gpurun_out/${T}_tiles.err; exit 1; }
cat gpurun_out/${T}_tiles.md
for r in 1 2; do
for lib in _C.so _C_ab.so; do
  KVEDGE_LIB=$lib timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_b_${lib}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "$lib $(python tools/bench_line.py gpurun_out/${T}_b_${lib}_$r.txt)"
done
done
