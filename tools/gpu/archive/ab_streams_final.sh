# A/B on HEAD: one stream, two streams (tiles tuned as concurrent copies), two streams (tuned alone)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 30 --warmup 5 --streams 1 2>/dev/null | grep metric | sed "s/^/{\"cfg\": \"s1\", \"r\": /; s/$/}/" >> gpurun_out/ab_streams_final.jsonl || exit $?
  timeout -k 10 150 python bench.py --steps 30 --warmup 5 --streams 2 2>/dev/null | grep metric | sed "s/^/{\"cfg\": \"s2\", \"r\": /; s/$/}/" >> gpurun_out/ab_streams_final.jsonl || exit $?
  KVEDGE_TUNE_CONCURRENT=0 timeout -k 10 150 python bench.py --steps 30 --warmup 5 --streams 2 2>/dev/null | grep metric | sed "s/^/{\"cfg\": \"s2-tune-alone\", \"r\": /; s/$/}/" >> gpurun_out/ab_streams_final.jsonl || exit $?
done
