# split-K as per-slice slabs (plain stores) + finalize: kernel tests, edge block, b1 profile
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3g}
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 > gpurun_out/${T}_edge.txt 2>&1 || exit $?
grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_edge.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_fwd1 -o fwd1 -- \
  python3 tools/profile_forward.py --batch 1 --reps 20 > gpurun_out/${T}_fwd1.log 2>&1 && \
python tools/profile_forward.py --summarize gpurun_out/${T}_fwd1/fwd1_kernel_trace.csv --reps 20 \
  > gpurun_out/${T}_fwd_b1.md
rc=$?
rm -rf gpurun_out/${T}_fwd1
head -30 gpurun_out/${T}_fwd_b1.md
exit $rc
