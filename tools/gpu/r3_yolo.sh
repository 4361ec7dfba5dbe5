# YOLOv8n per-op roofline (b192 slice of the b384 bench) + ResNet-50 cross-check of the op table
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/yolo_op_roofline_b192.md 2> gpurun_out/yolo_op_roofline.err && \
timeout -k 10 400 python -u tools/op_roofline.py --model resnet50 --batch 640 --streams 2 > gpurun_out/resnet_op_roofline_b640.md 2> gpurun_out/resnet_op_roofline.err
rc=$?
tail -n 4 gpurun_out/yolo_op_roofline_b192.md; tail -n 4 gpurun_out/resnet_op_roofline_b640.md
tail -n 3 gpurun_out/*.err
exit $rc
