# ResNet-50 b640 per-layer roofline (trace-matched) + large-batch cliff (b2048 / b2560, autotuned)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwd -o fwd -- python3 tools/profile_forward.py --batch 640 > gpurun_out/fwd.log 2>&1 && \
python tools/roofline_table.py gpurun_out/fwd/fwd_kernel_trace.csv --batch 640 > gpurun_out/roofline_b640.md
rc=$?; tail -n 3 gpurun_out/roofline_b640.md; [ $rc -ne 0 ] && exit $rc
for B in 2048 2560; do
  timeout -k 10 480 python -u bench.py --batch $B --steps 10 --warmup 3 --edge "" > gpurun_out/cliff_b$B.log 2>&1 || exit $?
  tail -n 1 gpurun_out/cliff_b$B.log | cut -c1-220
done
