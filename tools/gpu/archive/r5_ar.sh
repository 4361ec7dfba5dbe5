# Round 5 (ar): rocprofv3 kernel statistics of the final tree's headline bench (ResNet-50 b1280,
# two slices, one hipGraph per step; autotune and refine included in the trace)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ar}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o b -- python3 bench.py --steps 10 --warmup 3 --edge '' --yolo 0 > gpurun_out/${T}_bench.txt 2>gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
python3 tools/bench_line.py gpurun_out/${T}_bench.txt
f=$(ls gpurun_out/${T}_prof/*kernel_stats.csv | head -1); cp "$f" gpurun_out/${T}_kernel_stats.csv
rm -f gpurun_out/${T}_prof/*kernel_trace.csv
head -15 gpurun_out/${T}_kernel_stats.csv | cut -c1-200
