# Round 5 (c): v11 fused bottleneck -- numerics, model parity, bench A/B (KVEDGE_BNECK=0/1),
# in-graph layer table with it on.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5c}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "bneck" > gpurun_out/${T}_tk.txt 2>&1 || { tail -40 gpurun_out/${T}_tk.txt; exit 1; }
tail -2 gpurun_out/${T}_tk.txt
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_bench_config_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "resnet and not yolo" > gpurun_out/${T}_tm.txt 2>&1 || { tail -40 gpurun_out/${T}_tm.txt; exit 1; }
tail -2 gpurun_out/${T}_tm.txt
for i in 1 2; do
  KVEDGE_BNECK=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" --yolo 0 > gpurun_out/${T}_off$i.txt 2>&1 || { tail -20 gpurun_out/${T}_off$i.txt; exit 1; }
  echo "bneck off $i $(grep -o '"value": [0-9.]*' gpurun_out/${T}_off$i.txt | head -1)"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" --yolo 0 > gpurun_out/${T}_on$i.txt 2>&1 || { tail -20 gpurun_out/${T}_on$i.txt; exit 1; }
  echo "bneck on  $i $(grep -o '"value": [0-9.]*' gpurun_out/${T}_on$i.txt | head -1)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_gl2 -o gl \
  -- python3 tools/graph_layers.py run --streams 2 --labels gpurun_out/${T}_gl2_labels.json \
  > gpurun_out/${T}_gl2.log 2>&1 || { tail -20 gpurun_out/${T}_gl2.log; exit 1; }
python3 tools/graph_layers.py summarize gpurun_out/${T}_gl2 --labels gpurun_out/${T}_gl2_labels.json \
  > gpurun_out/${T}_graph_layers_s2.md 2>&1 || { tail -20 gpurun_out/${T}_graph_layers_s2.md; exit 1; }
head -4 gpurun_out/${T}_graph_layers_s2.md | tail -1
