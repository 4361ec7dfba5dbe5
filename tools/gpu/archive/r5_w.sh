# Round 5 (w): Detect stem 64 -> 144 as 80 + 64 (balanced split) vs 128 + 16: direct tests + YOLO A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5w}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "direct or every_tile or pair" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "yolo or Yolo" > gpurun_out/${T}_pytest_yolo.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_yolo.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest_yolo.txt
for r in 1 2; do
for sp in greedy balanced; do
  KVEDGE_DIRECT_SPLIT=$sp timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 5 > gpurun_out/${T}_yolo_${sp}_$r.txt 2>gpurun_out/${T}_yolo.err || { tail -20 gpurun_out/${T}_yolo.err; exit 1; }
  echo "split=$sp $(python -c "import json; d=json.loads(open('gpurun_out/${T}_yolo_${sp}_$r.txt').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
done
