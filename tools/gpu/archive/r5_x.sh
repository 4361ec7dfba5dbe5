# Round 5 (x): the neck's upsample + concat folded into h12 / h15 cv1 (conv_dual2 up2): kernel
# tests, the kernel test tier around duals, YOLO model tests, YOLO bench A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5x}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dual or tile_count or every_tile or canary" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "yolo or Yolo" > gpurun_out/${T}_pytest_yolo.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_yolo.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest_yolo.txt
for r in 1 2; do
for f in 0 1; do
  KVEDGE_YOLO_FUSE_UP=$f timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 5 > gpurun_out/${T}_yolo_up${f}_$r.txt 2>gpurun_out/${T}_yolo.err || { tail -20 gpurun_out/${T}_yolo.err; exit 1; }
  echo "fuse_up=$f $(python -c "import json; d=json.loads(open('gpurun_out/${T}_yolo_up${f}_$r.txt').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
done
