# YOLO Detect-branch pairs (3x3 + 1x1 fused, conv_direct C2 forms): tests, A/B, op roofline
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3j}
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "pair or direct" > gpurun_out/${T}_t1.txt 2>&1 || { tail -30 gpurun_out/${T}_t1.txt; exit 1; }
tail -1 gpurun_out/${T}_t1.txt
timeout -k 10 500 python -u -m pytest tests/test_models_gpu.py tests/test_bench_config_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/${T}_t2.txt 2>&1 || { tail -30 gpurun_out/${T}_t2.txt; exit 1; }
tail -1 gpurun_out/${T}_t2.txt
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_$i.txt 2>&1 || exit $?
  KVEDGE_YOLO_PAIR=0 timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_nopair_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/${T}_yolo_*.txt; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 \
  > gpurun_out/${T}_yolo_roofline_b192.md 2> gpurun_out/${T}_yolo_roofline.err || exit $?
grep "pair\|Forward" gpurun_out/${T}_yolo_roofline_b192.md
# edge serving batches: one vs two batch slices (engine.edge_streams)
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 --edge 8,32,64 > gpurun_out/${T}_edge2.txt 2>&1 || exit $?
KVEDGE_EDGE_STREAMS=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 --edge 8,32,64 > gpurun_out/${T}_edge1.txt 2>&1 || exit $?
for f in edge2 edge1; do echo "$f $(grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_$f.txt)"; done
