# Round 6 (c): y_sub (fused tails store only the stride-2 sample of y at the stage 1->2 and
# 2->3 boundaries) -- kernel + model tests, then the headline alternated KVEDGE_YSUB=1 / 0
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6c}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_bench_config_gpu.py -x -q --timeout 120 --timeout-method thread -k "ysub or tail or seam or resnet or dual" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2; do
for ys in 1 0; do
  KVEDGE_YSUB=$ys KVEDGE_BENCH_YOLO=0 KVEDGE_EDGE= timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 > gpurun_out/${T}_b_${ys}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "ysub=$ys $(python tools/bench_line.py gpurun_out/${T}_b_${ys}_$r.txt)"
done
done
