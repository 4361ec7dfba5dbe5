# Round 5 (v): headline A/B: tuner without (KVEDGE_TILE_LIMIT=108) / with the v12 edge family
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5v}
for r in 1 2; do
for lim in 108 0; do
  KVEDGE_TILE_LIMIT=$lim timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --edge "" --yolo 0 > gpurun_out/${T}_rn_${lim}_$r.txt 2>gpurun_out/${T}_rn.err || { tail -20 gpurun_out/${T}_rn.err; exit 1; }
  echo "limit=$lim $(python -c "import json; d=json.loads(open('gpurun_out/${T}_rn_${lim}_$r.txt').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
done
