# Round 5 (al): stage-2/3 seams (conv_seam) with y stored and the residual DMA'd non-temporal
# (_C.so) vs default policy (_C_ab.so, with the stage-1 tail change in both): seam tests, then
# the b1280 headline alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5al}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "seam or tail" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2 3; do
for lib in _C.so _C_ab.so; do
  KVEDGE_LIB=$lib timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge '' --yolo 0 > gpurun_out/${T}_b_${lib}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "$lib $(python tools/bench_line.py gpurun_out/${T}_b_${lib}_$r.txt)"
done
done
