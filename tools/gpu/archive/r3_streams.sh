# ResNet-50 slices x streams sweep on one box (autotuned per slice shape)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "1280 2" "1920 3" "1920 2" "2560 4"; do
  set -- $cfg
  timeout -k 10 420 python -u bench.py --batch $1 --streams $2 --steps 10 --warmup 3 --edge "" > gpurun_out/st_$1_$2.log 2>&1 || exit $?
  echo "b$1 s$2 $(tail -n 1 gpurun_out/st_$1_$2.log | grep -o '"value": [0-9.]*')" | tee -a gpurun_out/streams_sweep.txt
done
