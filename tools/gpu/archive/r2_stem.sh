# Stem ring: stem tests, then the bench + forward profile.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py -k "stem" > gpurun_out/pytest_stem.log 2>&1 && \
bash tools/gpu_check.sh bench fwd > gpurun_out/stem_steps.log 2>&1
rc=$?
tail -n 3 gpurun_out/pytest_stem.log
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'])"
grep stem gpurun_out/fwd_summary.md; head -1 gpurun_out/fwd_summary.md
exit $rc
