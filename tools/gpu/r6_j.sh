# Round 6 (j): the full default bench with the v14 tiles (117 256x256, 118 512x128) and the
# in-graph layer table: which layers pick which v14 tile
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6j}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_pp or (every_tile and 118) or (dual and 118) or (skinny and 118) or tile_count" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.txt 2>gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python tools/bench_line.py gpurun_out/${T}_bench.txt
d=gpurun_out/${T}_gl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
  python3 tools/graph_layers.py run --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
rm -rf $d
head -4 ${d}.md | tail -2
grep -c "pp:118" ${d}.md || true
