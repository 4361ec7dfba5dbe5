# Round 4: v9 seam kernel -- numerics, same-box bench A/B (KVEDGE_SEAM=1/0), b640 roofline
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4s}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "seam or tail" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for i in 1 2; do
  KVEDGE_SEAM=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench_seam$i.txt 2>&1 || exit $?
  KVEDGE_SEAM=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench_noseam$i.txt 2>&1 || exit $?
done
for f in bench_seam1 bench_noseam1 bench_seam2 bench_noseam2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${T}_$f.txt)"; done
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_fwd -o fwd -- python3 tools/profile_forward.py --batch 640 > gpurun_out/${T}_fwd.log 2>&1 && \
python tools/roofline_table.py gpurun_out/${T}_fwd/fwd_kernel_trace.csv --batch 640 > gpurun_out/${T}_roofline_b640.md
rc=$?; tail -n 3 gpurun_out/${T}_roofline_b640.md; exit $rc
