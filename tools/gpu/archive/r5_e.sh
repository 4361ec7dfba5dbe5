# Round 5 (e): module cold start (process start -> first inference, cold + warm tuner cache),
# the full default bench (headline + edge + YOLOv8n extra), the edited parity tests.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5e}
timeout -k 10 400 python -u tools/module_cold_start.py --model resnet50 --batch 64 --out gpurun_out/${T}_cold_start.json > gpurun_out/${T}_cold.txt 2>&1 || { tail -30 gpurun_out/${T}_cold.txt; exit 1; }
tail -1 gpurun_out/${T}_cold.txt
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.txt 2>&1 || { tail -30 gpurun_out/${T}_bench.txt; exit 1; }
grep '"metric"' gpurun_out/${T}_bench.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['extra'].get('edge'), d['extra'].get('yolov8n'), d['extra'].get('graph_refine'), d['extra'].get('prepare_s'))"
timeout -k 10 400 python -u -m pytest tests/test_bench_config_gpu.py tests/test_edge_config_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
