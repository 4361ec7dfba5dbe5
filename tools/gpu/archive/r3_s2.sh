# Round 3, session 2: full GPU tests + smoke, benches (ResNet with edge block, YOLO), split-K
# fixup A/B at the edge batches, b1 and b640 kernel traces (roofline table)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3e}
bash tools/gpu_check.sh $T tests smoke bench yolo || exit $?
KVEDGE_SK_FINALIZE=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 \
  > gpurun_out/${T}_edge_finalize.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_fwd1 -o fwd1 -- \
  python3 tools/profile_forward.py --batch 1 --reps 20 > gpurun_out/${T}_fwd1.log 2>&1 && \
python tools/profile_forward.py --summarize gpurun_out/${T}_fwd1/fwd1_kernel_trace.csv --reps 20 \
  > gpurun_out/${T}_fwd_b1.md || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_fwd -o fwd -- \
  python3 tools/profile_forward.py --batch 640 > gpurun_out/${T}_fwd640.log 2>&1 && \
python tools/roofline_table.py gpurun_out/${T}_fwd/fwd_kernel_trace.csv --batch 640 \
  > gpurun_out/${T}_roofline_b640.md
rc=$?
rm -rf gpurun_out/${T}_fwd1 gpurun_out/${T}_fwd
tail -n 2 gpurun_out/${T}_roofline_b640.md; head -12 gpurun_out/${T}_fwd_b1.md
exit $rc
