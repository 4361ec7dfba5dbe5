# Round 6 (l): persistent v14 forms (tiles 119 / 120): correctness (incl. > 256 tiles, two
# tiles per workgroup), then the probe of all four v14 tiles at b640 (eager and 2-concurrent)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6l}
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "conv_pp or (every_tile and (117 or 118 or 119 or 120)) or (dual and (117 or 118 or 119 or 120)) or (skinny and (117 or 118 or 119 or 120)) or tile_count" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 400 python -u tools/tile_probe.py --batch 640 --only s2.c1,s3.c1,s4.c3,s4.c1,s3.c3-nores,s2.c2,s3.c2,s4.c2,s2.c2s,s3.c2s,s4.c2s --tiles 80,117,118,119,120 > gpurun_out/${T}_tiles.md 2>&1 || { tail -20 gpurun_out/${T}_tiles.md; exit 1; }
grep "^|" gpurun_out/${T}_tiles.md
timeout -k 10 400 python -u tools/tile_probe.py --batch 640 --concurrent 2 --only s3.c1,s4.c1,s3.c2,s4.c2,s4.c3 --tiles 80,117,119 > gpurun_out/${T}_tiles_c2.md 2>&1 || { tail -20 gpurun_out/${T}_tiles_c2.md; exit 1; }
grep "^|" gpurun_out/${T}_tiles_c2.md
for lim in 0 117; do
  d=gpurun_out/${T}_gly_$lim
  KVEDGE_TILE_LIMIT=$lim timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
    python3 tools/graph_layers.py run --model yolov8n --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
  python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
  rm -rf $d
  echo "yolo limit=$lim $(head -4 ${d}.md | tail -1)"
done
