# Round 4 (u): YOLO stem2 fragment prefetch (b0 and b1 phases): numerics, op time, bench A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4u}
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_bench_config_gpu.py -x -q --timeout 150 --timeout-method thread -k "yolo or stem" > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for r in 1 2; do
  for lib in _C.so _C_ab.so; do
    KVEDGE_LIB=$lib timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_${lib}_$r.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo_${lib}_$r.txt; exit 1; }
    echo "$lib $r $(grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo_${lib}_$r.txt | head -1)"
  done
done
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/${T}_yolo_op_roofline_b192.md 2> gpurun_out/${T}_yolo.err || { tail -5 gpurun_out/${T}_yolo.err; exit 1; }
grep -E "\| 0 \||Forward" gpurun_out/${T}_yolo_op_roofline_b192.md
