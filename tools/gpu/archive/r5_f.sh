# Round 5 (f): NMS bucket sort -- numerics, phase probe + bucket/bitonic A/B, YOLO bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5f}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "nms or yolo" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 200 python -u tools/nms_probe.py --batch 256 > gpurun_out/${T}_nms_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_nms_probe.txt; exit 1; }
cat gpurun_out/${T}_nms_probe.txt | grep -v amdgpu.ids
for i in 1 2; do
  KVEDGE_STREAM_PRIO=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" --yolo 0 > gpurun_out/${T}_prio$i.txt 2>&1 || { tail -20 gpurun_out/${T}_prio$i.txt; exit 1; }
  echo "prio $i $(grep -o '"value": [0-9.]*' gpurun_out/${T}_prio$i.txt | head -1)"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" --yolo 0 > gpurun_out/${T}_base$i.txt 2>&1 || { tail -20 gpurun_out/${T}_base$i.txt; exit 1; }
  echo "base $i $(grep -o '"value": [0-9.]*' gpurun_out/${T}_base$i.txt | head -1)"
done
