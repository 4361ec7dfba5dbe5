# split-K + everything since the last full GPU pass: kernel/model tests, bench (edge block), b1/b64 profiles
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $P tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_block_gpu.py > gpurun_out/pytest_sk.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_sk.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwd1 -o fwd1 -- python3 tools/profile_forward.py --batch 1 --reps 20 > gpurun_out/fwd1.log 2>&1 && \
python tools/profile_forward.py --summarize gpurun_out/fwd1/fwd1_kernel_trace.csv --reps 20 > gpurun_out/fwd_b1.md && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwd64 -o fwd64 -- python3 tools/profile_forward.py --batch 64 --reps 20 > gpurun_out/fwd64.log 2>&1 && \
python tools/profile_forward.py --summarize gpurun_out/fwd64/fwd64_kernel_trace.csv --reps 20 > gpurun_out/fwd_b64.md
rc=$?
tail -n 1 gpurun_out/bench.log | cut -c1-300; grep -o '"edge": \[[^]]*\]' gpurun_out/bench.log
head -3 gpurun_out/fwd_b1.md; head -3 gpurun_out/fwd_b64.md
exit $rc
