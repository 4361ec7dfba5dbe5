# Frames-in ResNet stem: its tests, the model tests, ResNet bench.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_models_gpu.py > gpurun_out/stemf_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --profile gpurun_out/prof_resnet.json > gpurun_out/bench_prof.log 2>&1
rc=$?
tail -n 4 gpurun_out/stemf_tests.log; tail -n 1 gpurun_out/bench.log
exit $rc
