# Round 5 (ad): non-temporal residual loads in the v2/v7 (glds / xp) epilogues (_C.so; from the
# second run on gated to outputs > 64 MB) vs the
# default policy (_C_ab.so): GEMM-tile tests, then the full default bench (headline b1280,
# edge b1/b8/b64, YOLOv8n) alternated per library on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ad}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "every_tile or dual or res" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2; do
for lib in _C.so _C_ab.so; do
  KVEDGE_LIB=$lib timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_b_${lib}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "$lib $(python tools/bench_line.py gpurun_out/${T}_b_${lib}_$r.txt)"
done
done
