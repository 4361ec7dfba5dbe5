# Round 4 (y): v10 direct-epilogue forms with a residual (YOLO C2f bottleneck cv2): numerics,
# per-layer tile probe, same-box YOLO bench A/B (KVEDGE_DE_RES=0 refuses the new forms)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4y}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "direct or canary or tile_count or every_tile" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for sp in "192,160,160,16,16,3,1" "192,80,80,32,32,3,1" "192,40,40,64,64,3,1"; do
  echo "## $sp silu +res" >> gpurun_out/${T}_probe.txt; timeout -k 10 120 python3 tools/conv_probe.py --shape $sp --act silu --res --tiles 1,54,55,57,105,106 --iters 20 >> gpurun_out/${T}_probe.txt 2>&1 || { tail -5 gpurun_out/${T}_probe.txt; exit 1; }
  echo "## $sp silu (no res)" >> gpurun_out/${T}_probe.txt; timeout -k 10 120 python3 tools/conv_probe.py --shape $sp --act silu --tiles 105,106 --iters 20 >> gpurun_out/${T}_probe.txt 2>&1 || { tail -5 gpurun_out/${T}_probe.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/${T}_probe.txt
for r in 1 2; do
  for v in 1 0; do
    KVEDGE_DE_RES=$v timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_${v}_$r.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo_${v}_$r.txt; exit 1; }
    echo "DE_RES=$v run $r: $(grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo_${v}_$r.txt | head -1)"
  done
done
