set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_streams_gpu.py tests/test_bench_config_gpu.py > gpurun_out/t_streams.log 2>&1 || exit $?
for i in 1 2; do
for st in 1 2; do
timeout -k 10 120 python bench.py --steps 30 --warmup 5 --streams $st 2>/dev/null | grep metric >> gpurun_out/ab_streams.jsonl || exit $?
done; done
for st in 1 2; do
timeout -k 10 120 python bench.py --model yolov8n --steps 20 --warmup 3 --streams $st 2>/dev/null | grep metric >> gpurun_out/ab_streams.jsonl || exit $?
timeout -k 10 120 python bench.py --model yolov8n --batch 768 --steps 20 --warmup 3 --streams $st 2>/dev/null | grep metric >> gpurun_out/ab_streams.jsonl || exit $?
done
