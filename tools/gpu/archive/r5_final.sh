# Round 5 final: the whole GPU tier, smoke, the default bench (headline + edge + YOLOv8n),
# a same-box YOLOv8n A/B of the fused C2f, and the module cold start
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.txt 2>gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.txt | cut -c1-400
for r in 1 2; do
for c in 0 1; do
  KVEDGE_C2F=$c timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 5 > gpurun_out/${T}_yolo_c2f${c}_$r.txt 2>gpurun_out/${T}_yolo.err || { tail -20 gpurun_out/${T}_yolo.err; exit 1; }
  echo "c2f=$c $(python -c "import json; d=json.loads(open('gpurun_out/${T}_yolo_c2f${c}_$r.txt').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
done
timeout -k 10 600 python -u tools/module_cold_start.py --model resnet50 --batch 64 --out gpurun_out/${T}_cold_start.json > gpurun_out/${T}_cold.log 2>&1 || { tail -20 gpurun_out/${T}_cold.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_cold_start.json')); print([(r['run'], r['start_to_first_inference_s']) for r in d['runs']])"
