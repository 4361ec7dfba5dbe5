# A/B: autotuner without (KVEDGE_TILE_LIMIT=58) and with the v6 N-loop family
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "nloop or every_tile or tile_count or dual or canary" > gpurun_out/t_nloop.log 2>&1 || exit $?
for i in 1 2; do
for lim in 58 0; do
KVEDGE_TILE_LIMIT=$lim timeout -k 10 150 python bench.py --steps 30 --warmup 5 2>/dev/null | grep metric | sed "s/^/{\"tile_limit\": $lim, \"r\": /; s/$/}/" >> gpurun_out/ab_nloop.jsonl || exit $?
done; done
for lim in 58 0; do
KVEDGE_TILE_LIMIT=$lim timeout -k 10 150 python bench.py --model yolov8n --steps 20 --warmup 3 2>/dev/null | grep metric | sed "s/^/{\"tile_limit\": $lim, \"r\": /; s/$/}/" >> gpurun_out/ab_nloop.jsonl || exit $?
done
