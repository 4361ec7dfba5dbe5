# Round 6 (z11): v14 with B0 fragments kept in registers across the K-step (KV_PP_KEEPB: 24 fragment reads per K-step instead of 28) --
# correctness of tiles 117 / 119 (the persistent form), eager tile timing and the headline,
# alternated against the build without it (kvedge_amd/_C_kb0.so) on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z11}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "117 or 119 or pp or dual2" --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2; do
  for lib in _C.so _C_kb0.so; do
    KVEDGE_LIB=$lib timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --tiles 117,119 --only s3.c2,s4.c2,s3.c1,s3.c2s,s4.c2s,s4.c1 > gpurun_out/${T}_tiles_${lib}_$r.md 2>&1 || { tail -20 gpurun_out/${T}_tiles_${lib}_$r.md; exit 1; }
    echo "== $lib $r"; grep "^| s" gpurun_out/${T}_tiles_${lib}_$r.md
  done
done
for r in 1 2; do
  for lib in _C.so _C_kb0.so; do
    KVEDGE_LIB=$lib KVEDGE_BENCH_YOLO=0 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_b_${lib}_$r.txt 2>>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
    echo "$lib $r: $(python tools/bench_line.py gpurun_out/${T}_b_${lib}_$r.txt)"
  done
done
