# A/B: autotune timing tiles alone (KVEDGE_TUNE_CONCURRENT=0) vs as concurrent copies (=1)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for c in 0 1; do
KVEDGE_TUNE_CONCURRENT=$c timeout -k 10 150 python bench.py --steps 30 --warmup 5 2>/dev/null | grep metric | sed "s/^/{\"tune_conc\": $c, \"r\": /; s/$/}/" >> gpurun_out/ab_tune_conc.jsonl || exit $?
done; done
for c in 0 1; do
KVEDGE_TUNE_CONCURRENT=$c timeout -k 10 150 python bench.py --model yolov8n --steps 20 --warmup 3 2>/dev/null | grep metric | sed "s/^/{\"tune_conc\": $c, \"r\": /; s/$/}/" >> gpurun_out/ab_tune_conc.jsonl || exit $?
done
