# Round 6 final (second pass, on the tree as committed): GPU tier, smoke, default bench, bench
# kernel stats, in-graph layer tables (ResNet-50 b1280 / b64, YOLOv8n b512), module cold start
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6f2}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.txt 2>gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python tools/bench_line.py gpurun_out/${T}_bench.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o b -- python3 bench.py --steps 10 --warmup 3 --yolo 0 --edge "" > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
cp $(find gpurun_out/${T}_prof -name "b_kernel_stats.csv" | head -1) gpurun_out/${T}_bench_kernel_stats.csv
rm -rf gpurun_out/${T}_prof
for spec in "resnet50 0 0" "resnet50 64 1" "yolov8n 0 0"; do
  set -- $spec
  d=gpurun_out/${T}_gl_$1_$2
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
    python3 tools/graph_layers.py run --model $1 --batch $2 --streams $3 --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
  python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
  rm -rf $d
  echo "$1 b$2 $(grep 'Step wall' ${d}.md)"
done
timeout -k 10 600 python -u tools/module_cold_start.py --model resnet50 --batch 64 --out gpurun_out/${T}_cold_start.json > gpurun_out/${T}_cold.log 2>&1 || { tail -20 gpurun_out/${T}_cold.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_cold_start.json')); print([(r['run'], r['start_to_first_inference_s']) for r in d['runs']])"
