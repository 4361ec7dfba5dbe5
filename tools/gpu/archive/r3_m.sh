# stem12 pool lane remap A/B (_C_ab.so = previous stem12.hip) + synth counter paths + final benches
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3m}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "synth or stem or softmax" > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for i in 1 2; do
  timeout -k 10 200 python -u tools/stem_ab.py >> gpurun_out/${T}_stem.txt 2>&1 || exit $?
  KVEDGE_LIB=_C_ab.so timeout -k 10 200 python -u tools/stem_ab.py >> gpurun_out/${T}_stem.txt 2>&1 || exit $?
done
grep '^{' gpurun_out/${T}_stem.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.txt 2>&1 || exit $?
KVEDGE_LIB=_C_ab.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench_ab.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || exit $?
for f in bench bench_ab yolo; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${T}_$f.txt) $(grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_$f.txt)"; done
