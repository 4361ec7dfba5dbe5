# Round 4 (e): v10 direct-epilogue tiles (numerics, YOLO / ResNet A/B), deeper-residual seam
# forms (numerics + probe), then the seam PMC / b1 / op-roofline set of r4_d.sh
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4e}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "direct or canary or seam or tile_count or splitk or every_tile or pair or nms" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_de.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo_de.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo_de.txt | head -1
KVEDGE_TILE_LIMIT=105 timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_base.txt 2>&1 || { tail -5 gpurun_out/${T}_yolo_base.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_yolo_base.txt | head -1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_resnet.txt 2>&1 || { tail -5 gpurun_out/${T}_resnet.txt; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${T}_resnet.txt | head -1
timeout -k 10 300 python -u tools/seam_probe.py --batch 640 > gpurun_out/${T}_seam_probe.md 2>&1 || { cat gpurun_out/${T}_seam_probe.md; exit 1; }
cut -c1-700 gpurun_out/${T}_seam_probe.md
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/${T}_yolo_op_roofline_b192.md 2> gpurun_out/${T}_yolo.err || { tail -5 gpurun_out/${T}_yolo.err; exit 1; }
tail -n 4 gpurun_out/${T}_yolo_op_roofline_b192.md
bash tools/gpu/r4_pmc_seam.sh > gpurun_out/${T}_pmc.txt 2>&1 || { tail -20 gpurun_out/${T}_pmc.txt; exit 1; }
cut -c1-400 gpurun_out/pmc/summary_s3.md gpurun_out/pmc/summary_s2.md
