# Round 4: ResNet-50 micro-batched stage 1 (KVEDGE_MICROBATCH) re-checked on the final tree, same box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4mb}
for r in 1 2; do
  for mb in 0 160 320; do
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" --microbatch $mb > gpurun_out/${T}_${mb}_$r.txt 2>&1 || { tail -5 gpurun_out/${T}_${mb}_$r.txt; exit 1; }
    echo "microbatch $mb run $r: $(grep -o '"value": [0-9.]*' gpurun_out/${T}_${mb}_$r.txt | head -1)" | tee -a gpurun_out/${T}_ab.txt
  done
done
