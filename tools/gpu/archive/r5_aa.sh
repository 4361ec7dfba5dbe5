# Round 5 (aa): YOLO stem2 on 5 waves (one 32-pixel b1 block per wave) vs the 4-wave form
# (_C_ab.so): stem kernel tests, YOLO model tests, ISA lint, YOLO bench A/B on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5aa}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "stem or yolo or Yolo" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2 3; do
for lib in _C.so _C_ab.so; do
  KVEDGE_LIB=$lib timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 5 > gpurun_out/${T}_yolo_${lib}_$r.txt 2>gpurun_out/${T}_yolo.err || { tail -20 gpurun_out/${T}_yolo.err; exit 1; }
  echo "$lib $(python -c "import json; d=json.loads(open('gpurun_out/${T}_yolo_${lib}_$r.txt').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
done
