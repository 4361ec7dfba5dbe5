# Default bench batch 1280: bench-config parity test, then three fresh bench processes + b640 A/B.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_config_gpu.py > gpurun_out/pytest_b1280.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_b1280_$i.json > gpurun_out/bench_b1280_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --batch 640 --steps 30 --warmup 5 --json-out gpurun_out/bench_b640_$i.json > gpurun_out/bench_b640_$i.log 2>&1 || exit $?
done
tail -n 2 gpurun_out/pytest_b1280.log
for f in gpurun_out/bench_b1280_1 gpurun_out/bench_b640_1 gpurun_out/bench_b1280_2 gpurun_out/bench_b640_2; do
  python3 -c "import json; d=json.load(open('$f.json')); print('$f', d['value'], d['ms_per_step'], d['config']['global_batch'], d['extra']['build_s'])"
done
