# Round 5 (ao): YOLOv8n fused stem (frames) and fused C2f (x) read their last-use inputs
# non-temporal (_C.so) vs default policy (_C_ab.so): C2f / stem tests, YOLO bench alternated
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ao}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "c2f or stem2 or yolo" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2 3; do
for lib in _C.so _C_ab.so; do
  KVEDGE_LIB=$lib timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 5 > gpurun_out/${T}_y_${lib}_$r.txt 2>gpurun_out/${T}_y.err || { tail -20 gpurun_out/${T}_y.err; exit 1; }
  echo "$lib $(python tools/bench_line.py gpurun_out/${T}_y_${lib}_$r.txt)"
done
done
