# Round 5 (n): default bench (ResNet-50 headline + edge block + YOLOv8n extra) with the v12 family
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5n}
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.txt 2>gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.txt
