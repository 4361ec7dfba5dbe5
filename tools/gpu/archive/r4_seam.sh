# Round 4: v9 seam kernel + edge head -- numerics, same-box bench A/B (KVEDGE_SEAM=1/0,
# KVEDGE_FUSE_HEAD=0/1 for the edge points), b640 roofline
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4s}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "seam or tail or pooled_fc or pde or every_tile or canary or dual" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u -m pytest tests/test_edge_config_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${T}_edge_t.txt 2>&1 || { tail -40 gpurun_out/${T}_edge_t.txt; exit 1; }
tail -1 gpurun_out/${T}_edge_t.txt
for i in 1 2; do
  KVEDGE_SEAM=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench_seam$i.txt 2>&1 || exit $?
  KVEDGE_SEAM=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench_noseam$i.txt 2>&1 || exit $?
done
KVEDGE_TILE_LIMIT=86 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench_nopde.txt 2>&1 || exit $?
for f in bench_seam1 bench_noseam1 bench_seam2 bench_noseam2 bench_nopde; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${T}_$f.txt)"; done
KVEDGE_FUSE_HEAD=0 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 > gpurun_out/${T}_edge_head0.txt 2>&1 || exit $?
KVEDGE_FUSE_HEAD=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 > gpurun_out/${T}_edge_head1.txt 2>&1 || exit $?
for f in edge_head0 edge_head1; do echo "$f $(grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_$f.txt)"; done
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_fwd -o fwd -- python3 tools/profile_forward.py --batch 640 > gpurun_out/${T}_fwd.log 2>&1 && \
python tools/roofline_table.py gpurun_out/${T}_fwd/fwd_kernel_trace.csv --batch 640 > gpurun_out/${T}_roofline_b640.md
rc=$?; tail -n 3 gpurun_out/${T}_roofline_b640.md; exit $rc
