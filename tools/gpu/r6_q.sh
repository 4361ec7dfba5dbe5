# Round 6 (q): ResNet stage-2 entry 3x3/2 with the new ReLU direct form (tile probe, alone and
# two concurrent); NMS at b192; YOLOv8n in-graph table with per-op kernel counts from the
# trace (floors for every op); v11 fused bottleneck at the edge batches (on / off)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6q}
timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --only s2.c2s,s2.c2 > gpurun_out/${T}_tiles_c1.md 2>&1 || { tail -20 gpurun_out/${T}_tiles_c1.md; exit 1; }
timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --only s2.c2s --concurrent 2 > gpurun_out/${T}_tiles_c2.md 2>&1 || { tail -20 gpurun_out/${T}_tiles_c2.md; exit 1; }
timeout -k 10 300 python -u tools/nms_probe.py --batch 192 > gpurun_out/${T}_nms192.txt 2>&1 || { tail -20 gpurun_out/${T}_nms192.txt; exit 1; }
d=gpurun_out/${T}_gly
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
  python3 tools/graph_layers.py run --model yolov8n --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
rm -rf $d
head -4 ${d}.md | tail -1
timeout -k 10 600 python -u tools/edge_ab.py --arms "KVEDGE_BNECK=0;KVEDGE_BNECK=1" --batches 8,64 --rounds 2 > gpurun_out/${T}_bneck_edge.jsonl 2>&1 || { tail -20 gpurun_out/${T}_bneck_edge.jsonl; exit 1; }
grep summary gpurun_out/${T}_bneck_edge.jsonl
