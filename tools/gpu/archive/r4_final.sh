# Round 4 tree: all GPU tests + smoke, then the benches (ResNet-50 with the edge block, YOLOv8n)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4z}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || exit $?
for f in bench yolo; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${T}_$f.txt) $(grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_$f.txt)"; done
