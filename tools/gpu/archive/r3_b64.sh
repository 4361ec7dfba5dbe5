# ResNet-50 edge batch 64: kernel table of one graph step (rocprofv3) + YOLO b192 op roofline
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3i}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_fwd64 -o fwd64 -- \
  python3 tools/profile_forward.py --batch 64 --reps 20 > gpurun_out/${T}_fwd64.log 2>&1 && \
python tools/profile_forward.py --summarize gpurun_out/${T}_fwd64/fwd64_kernel_trace.csv --reps 20 \
  > gpurun_out/${T}_fwd_b64.md || exit $?
rm -rf gpurun_out/${T}_fwd64
head -40 gpurun_out/${T}_fwd_b64.md
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 \
  > gpurun_out/${T}_yolo_roofline_b192.md 2> gpurun_out/${T}_yolo_roofline.err || exit $?
tail -4 gpurun_out/${T}_yolo_roofline_b192.md
