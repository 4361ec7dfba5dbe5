# Round 4 (h): v10 tile 2 (single patch buffer, 4 waves, 2 workgroups per CU): numerics,
# per-layer tile probe, YOLO bench + op roofline, ResNet bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4h}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "direct or canary or tile_count or every_tile or pair" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for sp in "192,80,80,64,128,3,1 silu" "192,80,80,64,16,3,1 silu" "640,56,56,64,64,3,1 relu" "192,80,80,32,32,3,1 silu" "192,40,40,64,64,3,1 silu" "192,160,160,32,64,3,2 silu"; do set -- $sp
  echo "## $1 $2" >> gpurun_out/${T}_probe.txt; timeout -k 10 120 python3 tools/conv_probe.py --shape $1 --act $2 --tiles 54,55,105,106,107 --iters 20 >> gpurun_out/${T}_probe.txt 2>&1 || { tail -5 gpurun_out/${T}_probe.txt; exit 1; }
done
for sp in "640,28,28,128,128,3,1 relu" "192,20,20,128,128,3,1 silu" "192,40,40,128,128,3,2 silu"; do set -- $sp
  echo "## $1 $2" >> gpurun_out/${T}_probe.txt; timeout -k 10 120 python3 tools/conv_probe.py --shape $1 --act $2 --tiles 7,24,29,55,76,83,105 --iters 20 >> gpurun_out/${T}_probe.txt 2>&1 || { tail -5 gpurun_out/${T}_probe.txt; exit 1; }
done
cat gpurun_out/${T}_probe.txt
timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo.txt | head -1
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/${T}_yolo_op_roofline_b192.md 2> gpurun_out/${T}_yolo.err || { tail -5 gpurun_out/${T}_yolo.err; exit 1; }
tail -n 4 gpurun_out/${T}_yolo_op_roofline_b192.md
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_resnet.txt 2>&1 || { tail -5 gpurun_out/${T}_resnet.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_resnet.txt | head -1
