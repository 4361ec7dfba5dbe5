# Round 5 final (late): the whole GPU tier, smoke, the default bench (headline + edge + YOLOv8n)
# and the module cold start, on the tree as committed
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.txt 2>gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python tools/bench_line.py gpurun_out/${T}_bench.txt
timeout -k 10 600 python -u tools/module_cold_start.py --model resnet50 --batch 64 --out gpurun_out/${T}_cold_start.json > gpurun_out/${T}_cold.log 2>&1 || { tail -20 gpurun_out/${T}_cold.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_cold_start.json')); print([(r['run'], r['start_to_first_inference_s']) for r in d['runs']])"
