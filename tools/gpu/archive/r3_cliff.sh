# Large-batch cliff check: autotuned bench at b1280 / b2048 / b2560 on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for B in 1280 2048 2560; do
  timeout -k 10 420 python -u bench.py --batch $B --steps 10 --warmup 3 --edge "" > gpurun_out/cliff_b$B.log 2>&1 || exit $?
  tail -n 1 gpurun_out/cliff_b$B.log | cut -c1-200
done
