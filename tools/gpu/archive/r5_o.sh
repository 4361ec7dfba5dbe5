# Round 5 (o): v13 fused C2f -- kernel tests, YOLO model tests, YOLO bench A/B (KVEDGE_C2F=0/1)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5o}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "c2f16" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "yolo or Yolo" > gpurun_out/${T}_pytest_yolo.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_yolo.txt; exit 1; }
tail -2 gpurun_out/${T}_pytest_yolo.txt
for r in 1 2; do
for c in 0 1; do
  KVEDGE_C2F=$c timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 5 > gpurun_out/${T}_yolo_c2f$c.txt 2>gpurun_out/${T}_yolo_c2f$c.err || { tail -20 gpurun_out/${T}_yolo_c2f$c.err; exit 1; }
  echo "c2f=$c $(python -c "import json,sys; d=json.loads(open('gpurun_out/${T}_yolo_c2f$c.txt').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
done
