# Round 6 (e): y_sub with the division-free pixel walk in the stream tail: kernel test, then
# in-graph per-layer tables KVEDGE_YSUB=1 vs 0
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6e}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "ysub" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for ys in 1 0; do
  d=gpurun_out/${T}_gl_$ys
  KVEDGE_YSUB=$ys timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
    python3 tools/graph_layers.py run --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
  python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
  rm -rf $d
  head -4 ${d}.md | tail -2
  grep -E "^\| (7|9|16|18) \|" ${d}.md | cut -d'|' -f2,3,6,9
done
