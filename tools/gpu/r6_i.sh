# Round 6 (i): v14 schedule variants (DMA placement, MFMA-cluster priority): correctness of
# each build, then the tile-117 probe alternated over the builds
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6i}
for lib in _C.so _C_d0.so _C_d2.so _C_p0.so; do
  KVEDGE_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_pp" > gpurun_out/${T}_pytest_$lib.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_$lib.txt; exit 1; }
  echo "$lib $(tail -1 gpurun_out/${T}_pytest_$lib.txt)"
done
for r in 1 2; do
for lib in _C.so _C_d0.so _C_d2.so _C_p0.so; do
  KVEDGE_LIB=$lib timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --only s3.c2,s4.c2,s3.c2s,s4.c1,s4.c3,s3.c1,s2.c2,s2.c1,s2.c2s --tiles 117,118 > gpurun_out/${T}_t_${lib}_$r.md 2>&1 || { tail -20 gpurun_out/${T}_t_${lib}_$r.md; exit 1; }
  echo "$lib r$r $(grep '^| s' gpurun_out/${T}_t_${lib}_$r.md | awk -F'|' '{printf "%s=%s ", $2, $3}')"
done
done
