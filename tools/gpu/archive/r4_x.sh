# Round 4 (x): rocprofv3 kernel trace of the bench configs (autotuned, hipGraph, 2 streams):
# ResNet-50 b1280 and YOLOv8n b384, per-kernel table of the measured replays.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4x}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_rn -o rn -- python3 tools/profile_forward.py --model resnet50 --batch 1280 --streams 2 --reps 3 > gpurun_out/${T}_rn.log 2>&1 && \
python3 tools/profile_forward.py --summarize "$(ls gpurun_out/${T}_rn/*/rn_kernel_trace.csv gpurun_out/${T}_rn/rn_kernel_trace.csv 2>/dev/null | head -1)" --reps 3 > gpurun_out/${T}_resnet50_b1280_kernels.md && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_yo -o yo -- python3 tools/profile_forward.py --model yolov8n --batch 384 --streams 2 --reps 3 > gpurun_out/${T}_yo.log 2>&1 && \
python3 tools/profile_forward.py --summarize "$(ls gpurun_out/${T}_yo/*/yo_kernel_trace.csv gpurun_out/${T}_yo/yo_kernel_trace.csv 2>/dev/null | head -1)" --reps 3 > gpurun_out/${T}_yolov8n_b384_kernels.md && \
head -3 gpurun_out/${T}_resnet50_b1280_kernels.md gpurun_out/${T}_yolov8n_b384_kernels.md
