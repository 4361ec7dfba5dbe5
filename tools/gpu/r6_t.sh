# Round 6 (t): 16-wave NMS (1024 threads per image) -- NMS tests, probe at b192 / b256,
# YOLOv8n bench; YOLOv8n in-graph table with per-op kernel counts (separator pass)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6t}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "nms or yolo" --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for b in 192 256; do
timeout -k 10 300 python -u tools/nms_probe.py --batch $b > gpurun_out/${T}_nms$b.txt 2>&1 || { tail -20 gpurun_out/${T}_nms$b.txt; exit 1; }
grep -E "max over|diag 0" gpurun_out/${T}_nms$b.txt
done
d=gpurun_out/${T}_gly
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
  python3 tools/graph_layers.py run --model yolov8n --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
rm -rf $d
head -4 ${d}.md | tail -1
KVEDGE_EDGE= timeout -k 10 600 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/${T}_yolo.txt 2>gpurun_out/${T}_yolo.err || { tail -20 gpurun_out/${T}_yolo.err; exit 1; }
python tools/bench_line.py gpurun_out/${T}_yolo.txt
