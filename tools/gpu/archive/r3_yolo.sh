# YOLOv8n per-op roofline (b192 slice of the b384 bench) + ResNet-50 cross-check of the op table
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/yolo_op_roofline_b192.md 2> gpurun_out/yolo_op_roofline.err && \
timeout -k 10 400 python -u tools/op_roofline.py --model resnet50 --batch 640 --streams 2 > gpurun_out/resnet_op_roofline_b640.md 2> gpurun_out/resnet_op_roofline.err
rc=$?
[ $rc -eq 0 ] && timeout -k 10 300 python -u tools/blas_ceiling.py --batch 640 > gpurun_out/blas_ceiling_b640.md 2>&1; rc=$?
cat gpurun_out/blas_ceiling_b640.md | tail -16
tail -n 4 gpurun_out/yolo_op_roofline_b192.md; tail -n 4 gpurun_out/resnet_op_roofline_b640.md
tail -n 3 gpurun_out/*.err
exit $rc
