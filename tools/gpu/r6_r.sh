# Round 6 (r): after removing bneck_fused and the full-rank NMS sort -- the GPU tier, the NMS
# probe at b192 / b256, and the default bench (headline + edge + YOLOv8n)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6r}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.txt
for b in 192 256; do
timeout -k 10 300 python -u tools/nms_probe.py --batch $b > gpurun_out/${T}_nms$b.txt 2>&1 || { tail -20 gpurun_out/${T}_nms$b.txt; exit 1; }
grep -E "max over|diag 0" gpurun_out/${T}_nms$b.txt
done
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.txt 2>gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python tools/bench_line.py gpurun_out/${T}_bench.txt
# stem12 PMC (three counter passes, each its own run) -- VERDICT r5 next 6: VALU- or DMA-bound?
timeout -k 10 400 bash tools/pmc_cmd.sh gpurun_out/${T}_stem_pmc tools/stem_probe.py --batch 640 --reps 3 > /dev/null 2>&1 || { echo "stem pmc failed"; exit 1; }
grep -E "stem12|kernel" gpurun_out/${T}_stem_pmc/summary.txt | head -5
