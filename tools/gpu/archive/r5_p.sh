# Round 5 (p): in-graph tables of the YOLOv8n bench step and the ResNet-50 b1280 bench step
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5p}
run() {  # tag model batch streams
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_$1 -o gl \
    -- python3 tools/graph_layers.py run --model $2 --batch $3 --streams $4 --reps 20 --labels gpurun_out/${T}_$1_labels.json \
    > gpurun_out/${T}_$1.log 2>&1 || { tail -20 gpurun_out/${T}_$1.log; return 1; }
  python3 tools/graph_layers.py summarize gpurun_out/${T}_$1 --reps 20 --labels gpurun_out/${T}_$1_labels.json \
    > gpurun_out/${T}_$1.md 2>&1 || { tail -20 gpurun_out/${T}_$1.md; return 1; }
  head -4 gpurun_out/${T}_$1.md | tail -1
  rm -rf gpurun_out/${T}_$1
}
run yolo_b512 yolov8n 512 2 && run rn_b1280 resnet50 1280 2
