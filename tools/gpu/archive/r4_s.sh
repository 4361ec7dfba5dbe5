# Round 4 (s): seams at edge batches: the default gate (256 128-row workgroups) vs 64
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4s2}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_edge_config_gpu.py -x -q --timeout 150 --timeout-method thread -k "seam or edge" > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for r in 1 2; do
  for g in 256 64; do
    KVEDGE_SEAM_MIN_WGS=$g timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --edge "8,64" > gpurun_out/${T}_edge_${g}_$r.txt 2>&1 || { tail -5 gpurun_out/${T}_edge_${g}_$r.txt; exit 1; }
    echo "gate $g run $r: $(grep -o '"edge": .*' gpurun_out/${T}_edge_${g}_$r.txt | cut -c1-300)"
  done
done
