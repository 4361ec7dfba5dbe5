# Edge-size batch rows (1/8/64) for both models + YOLOv8n b384 PMC passes (HBM bytes per kernel).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -f gpurun_out/sweep_edge.jsonl
timeout -k 10 400 python tools/batch_sweep.py --configs "1:0:0,8:0:0,64:0:0,640:0:0" --steps 30 \
    --out gpurun_out/sweep_edge.jsonl > gpurun_out/sweep_edge_resnet.log 2>&1 && \
timeout -k 10 400 python tools/batch_sweep.py --model yolov8n --configs "1:0:0,8:0:0,64:0:0,384:0:0" \
    --steps 20 --out gpurun_out/sweep_edge.jsonl > gpurun_out/sweep_edge_yolo.log 2>&1 && \
timeout -k 10 600 bash tools/pmc_cmd.sh gpurun_out/pmc_yolo tools/profile_forward.py --model yolov8n \
    --batch 384 --reps 2 > gpurun_out/pmc_yolo.log 2>&1
rc=$?
cat gpurun_out/sweep_edge.jsonl; tail -3 gpurun_out/pmc_yolo.log
exit $rc
