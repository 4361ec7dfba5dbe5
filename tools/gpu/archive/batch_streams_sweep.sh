# Two-stream bench at several per-GPU batches (slices of batch/2)
set -o pipefail
mkdir -p gpurun_out
for b in 1024 1280 1536 2048 1280; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --batch $b 2>/dev/null | grep metric >> gpurun_out/batch_streams.jsonl || exit $?
done
