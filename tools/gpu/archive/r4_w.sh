# Round 4 (w): autotune refine iterations 20 (default) vs 60, ResNet-50 bench, alternating
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4w}
for r in 1 2; do
  for it in 20 60; do
    KVEDGE_AUTOTUNE_REFINE_ITERS=$it timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_resnet_${it}_$r.txt 2>&1 || { tail -5 gpurun_out/${T}_resnet_${it}_$r.txt; exit 1; }
    echo "refine $it run $r: $(grep -o '"value": [0-9.]*' gpurun_out/${T}_resnet_${it}_$r.txt | head -1)"
  done
done
