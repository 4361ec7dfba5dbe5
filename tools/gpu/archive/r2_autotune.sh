# Autotune stability: three fresh bench processes on one box + one forward profile.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --json-out gpurun_out/bench_at$i.json > gpurun_out/bench_at$i.log 2>&1 || exit $?
done
bash tools/gpu_check.sh fwd > /dev/null 2>&1
rc=$?
for i in 1 2 3; do python3 -c "import json; d=json.load(open('gpurun_out/bench_at$i.json')); print(d['value'], d['ms_per_step'], d['extra']['build_s'])"; done
head -22 gpurun_out/fwd_summary.md
exit $rc
