# Round-3 baseline on a fresh box: headline bench + ResNet-50 b640 per-layer roofline.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
(command -v amd-smi >/dev/null && amd-smi list --json > gpurun_out/amdsmi_list.json 2>/dev/null; true) && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwd -o fwd -- python3 tools/profile_forward.py --batch 640 > gpurun_out/fwd.log 2>&1 && \
python tools/roofline_table.py gpurun_out/fwd/fwd_kernel_trace.csv --batch 640 > gpurun_out/roofline_b640.md
rc=$?
tail -n 1 gpurun_out/bench.log | cut -c1-300
tail -n 3 gpurun_out/roofline_b640.md
exit $rc
