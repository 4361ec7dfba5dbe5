# Round 6 (u): v15 256 x 160 tiles (YOLO Detect stems, N = 144) -- correctness, then YOLOv8n
# bench with / without them (KVEDGE_TILE_LIMIT=121 hides the family from the tuner),
# alternated on one box, and the in-graph table with them
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6u}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "121 or 122 or tile_count" --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2; do
  for lim in 0 121; do
    KVEDGE_TILE_LIMIT=$lim KVEDGE_EDGE= timeout -k 10 600 python -u bench.py --model yolov8n --steps 20 --warmup 5 > gpurun_out/${T}_y_${lim}_$r.txt 2>>gpurun_out/${T}_y.err || { tail -20 gpurun_out/${T}_y.err; exit 1; }
    echo "limit=$lim $r: $(python tools/bench_line.py gpurun_out/${T}_y_${lim}_$r.txt)"
  done
done
d=gpurun_out/${T}_gly
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
  python3 tools/graph_layers.py run --model yolov8n --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
rm -rf $d
grep -E "144|Step wall" ${d}.md | cut -c1-160
