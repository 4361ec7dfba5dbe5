# Round 4 (d): seam PMC; b1 edge forward profile; YOLOv8n + ResNet-50 per-op rooflines
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k seam > gpurun_out/r4d_seamtest.log 2>&1 || { tail -30 gpurun_out/r4d_seamtest.log; exit 1; }
tail -2 gpurun_out/r4d_seamtest.log
timeout -k 10 300 python -u tools/seam_probe.py --batch 640 > gpurun_out/r4d_seam_probe_b640.md 2> gpurun_out/r4d_probe.err || { tail -5 gpurun_out/r4d_probe.err; exit 1; }
cat gpurun_out/r4d_seam_probe_b640.md | cut -c1-600
bash tools/gpu/r4_pmc_seam.sh > gpurun_out/r4d_pmc.txt 2>&1 || { tail -20 gpurun_out/r4d_pmc.txt; exit 1; }
cat gpurun_out/pmc/summary_s3.md gpurun_out/pmc/summary_s2.md | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4d_b1 -o b1 -- python3 tools/profile_forward.py --batch 1 --reps 20 > gpurun_out/r4d_b1.log 2>&1 && \
python3 tools/profile_forward.py --summarize gpurun_out/r4d_b1/b1_kernel_trace.csv --reps 20 > gpurun_out/r4d_b1_forward.md 2>&1 || exit $?
head -30 gpurun_out/r4d_b1_forward.md
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 > gpurun_out/r4d_yolo_op_roofline_b192.md 2> gpurun_out/r4d_yolo.err || { tail -5 gpurun_out/r4d_yolo.err; exit 1; }
tail -n 4 gpurun_out/r4d_yolo_op_roofline_b192.md
timeout -k 10 400 python -u tools/op_roofline.py --model resnet50 --batch 640 --streams 2 > gpurun_out/r4d_resnet_op_roofline_b640.md 2> gpurun_out/r4d_resnet.err || { tail -5 gpurun_out/r4d_resnet.err; exit 1; }
tail -n 4 gpurun_out/r4d_resnet_op_roofline_b640.md
