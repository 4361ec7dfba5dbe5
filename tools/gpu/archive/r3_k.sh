# DE epilogue (residual up front, bias via LDS: counted waits between stores) A/B against
# _C_ab.so (previous epilogue); YOLO Detect pairs on/off; edge streams 2 vs 1; full tests
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3k}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_bench_config_gpu.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_rn_$i.txt 2>&1 || exit $?
  KVEDGE_LIB=_C_ab.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_rn_ab_$i.txt 2>&1 || exit $?
done
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || exit $?
KVEDGE_YOLO_PAIR=0 timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_nopair.txt 2>&1 || exit $?
KVEDGE_LIB=_C_ab.so KVEDGE_YOLO_PAIR=0 timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_ab_nopair.txt 2>&1 || exit $?
for f in gpurun_out/${T}_rn_*.txt gpurun_out/${T}_yolo*.txt; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 --edge 1,8,32,64 > gpurun_out/${T}_edge2.txt 2>&1 || exit $?
KVEDGE_EDGE_STREAMS=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 --edge 32,64 > gpurun_out/${T}_edge1.txt 2>&1 || exit $?
for f in edge2 edge1; do echo "$f $(grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_$f.txt)"; done
