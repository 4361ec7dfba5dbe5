# Round 4 (l): v10 tile 3 (two channel blocks per wave: half the LDS fragment bytes per FLOP)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4l}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "direct or canary or tile_count or every_tile" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for sp in "192,80,80,64,128,3,1 silu" "640,56,56,64,64,3,1 relu" "192,40,40,64,64,3,1 silu" "192,160,160,32,64,3,2 silu" "192,80,80,64,128,3,2 silu"; do set -- $sp
  for d in 0 7; do
    echo "## $1 $2 diag=$d" >> gpurun_out/${T}_probe.txt
    KVEDGE_DIRECT_DIAG=$d timeout -k 10 120 python3 tools/conv_probe.py --shape $1 --act $2 --tiles 54,105,107,108 --iters 20 >> gpurun_out/${T}_probe.txt 2>&1 || { tail -5 gpurun_out/${T}_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/${T}_probe.txt
timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo.txt | head -1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_resnet.txt 2>&1 || { tail -5 gpurun_out/${T}_resnet.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_resnet.txt | head -1
