# bench + b640 roofline + edge-batch kernel profiles (b1, b64)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "even_pixels or tail_fused or dual_fused" > gpurun_out/pytest_ys2.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwd -o fwd -- python3 tools/profile_forward.py --batch 640 > gpurun_out/fwd.log 2>&1 && \
python tools/roofline_table.py gpurun_out/fwd/fwd_kernel_trace.csv --batch 640 > gpurun_out/roofline_b640.md && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwd1 -o fwd1 -- python3 tools/profile_forward.py --batch 1 --reps 20 > gpurun_out/fwd1.log 2>&1 && \
python tools/profile_forward.py --summarize gpurun_out/fwd1/fwd1_kernel_trace.csv --reps 20 > gpurun_out/fwd_b1.md && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwd64 -o fwd64 -- python3 tools/profile_forward.py --batch 64 --reps 20 > gpurun_out/fwd64.log 2>&1 && \
python tools/profile_forward.py --summarize gpurun_out/fwd64/fwd64_kernel_trace.csv --reps 20 > gpurun_out/fwd_b64.md
rc=$?
tail -n 1 gpurun_out/bench.log | cut -c1-300; grep -o '"edge": \[[^]]*\]' gpurun_out/bench.log
tail -n 2 gpurun_out/roofline_b640.md; head -3 gpurun_out/fwd_b1.md; head -3 gpurun_out/fwd_b64.md
exit $rc
