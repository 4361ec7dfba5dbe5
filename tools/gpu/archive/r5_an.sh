# Round 5 (an): direct-family patch DMAs non-temporal when the input exceeds half the Infinity
# Cache (_C.so) vs default policy (_C_ab.so): direct / YOLO tests, then the full bench
# alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5an}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "direct or yolo or Yolo" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2; do
for lib in _C.so _C_ab.so; do
  KVEDGE_LIB=$lib timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_b_${lib}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "$lib $(python tools/bench_line.py gpurun_out/${T}_b_${lib}_$r.txt)"
done
done
