# same-box A/B: fused YOLO b0+b1 on / off (bench b384), op roofline with the fused stem, then PMC passes
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for F in 0 1 0 1; do
  KVEDGE_YOLO_FUSE_B1=$F timeout -k 10 300 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/ab_ys2_$F.log 2>&1 || exit $?
  echo "fuse=$F $(tail -n 1 gpurun_out/ab_ys2_$F.log | grep -o '"value": [0-9.]*')" | tee -a gpurun_out/ab_ys2.txt
done
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/yolo_op_roofline_b192_v4.md 2> gpurun_out/yolo_op_roofline.err || exit $?
head -6 gpurun_out/yolo_op_roofline_b192_v4.md | tail -2; grep "Forward" gpurun_out/yolo_op_roofline_b192_v4.md
bash tools/gpu/r3_pmc_direct.sh
