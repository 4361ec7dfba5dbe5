# A/B: fused stage-1 tails on the 32x32x16 (default) vs the 16x16x32 MFMA forms
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for m in 0 1; do
KVEDGE_TAIL_MF16=$m timeout -k 10 150 python bench.py --steps 30 --warmup 5 2>/dev/null | grep metric | sed "s/^/{\"tail_mf16\": $m, \"r\": /; s/$/}/" >> gpurun_out/ab_tail_mf16.jsonl || exit $?
done; done
for m in 0 1; do
KVEDGE_TAIL_MF16=$m timeout -k 10 150 python bench.py --steps 30 --warmup 5 --streams 1 2>/dev/null | grep metric | sed "s/^/{\"tail_mf16\": $m, \"r\": /; s/$/}/" >> gpurun_out/ab_tail_mf16.jsonl || exit $?
done
