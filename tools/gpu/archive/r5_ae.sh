# Round 5 (ae): the eager per-op rooflines the round-4 review set targets on (ResNet-50 one b640
# slice of 1280; YOLOv8n one b192 slice), on this round's kernels
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ae}
timeout -k 10 400 python -u tools/op_roofline.py --model resnet50 --batch 640 --streams 2 > gpurun_out/${T}_rn_op_roofline_b640.md 2> gpurun_out/${T}_rn.err || { tail -5 gpurun_out/${T}_rn.err; exit 1; }
grep -n "Forward" gpurun_out/${T}_rn_op_roofline_b640.md
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/${T}_yolo_op_roofline_b192.md 2> gpurun_out/${T}_yolo.err || { tail -5 gpurun_out/${T}_yolo.err; exit 1; }
grep -n "Forward" gpurun_out/${T}_yolo_op_roofline_b192.md
