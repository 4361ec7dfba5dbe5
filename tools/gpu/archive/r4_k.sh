# Round 4 (k): DE stores as 16-B half-wave-exchanged pairs vs the 4 x 8-B form (diag bit 3)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4k}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "direct or canary" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for sp in "192,80,80,64,128,3,1 silu" "640,56,56,64,64,3,1 relu" "192,80,80,64,16,3,1 silu" "640,28,28,128,128,3,1 relu"; do set -- $sp
  for d in 0 8 1 0; do
    echo "## $1 $2 diag=$d" >> gpurun_out/${T}_diag.txt
    KVEDGE_DIRECT_DIAG=$d timeout -k 10 120 python3 tools/conv_probe.py --shape $1 --act $2 --tiles 105,107 --iters 20 >> gpurun_out/${T}_diag.txt 2>&1 || { tail -5 gpurun_out/${T}_diag.txt; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/${T}_diag.txt
timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo.txt | head -1
