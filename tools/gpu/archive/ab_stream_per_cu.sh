# A/B under the two-stream bench: persistent v3 streaming kernel workgroups per CU cap
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for c in 0 2 1; do
if [ $c = 0 ]; then unset KVEDGE_STREAM_PER_CU; else export KVEDGE_STREAM_PER_CU=$c; fi
timeout -k 10 150 python bench.py --steps 30 --warmup 5 2>/dev/null | grep metric | sed "s/^/{\"per_cu\": $c, \"r\": /; s/$/}/" >> gpurun_out/ab_stream_per_cu.jsonl || exit $?
done; done
