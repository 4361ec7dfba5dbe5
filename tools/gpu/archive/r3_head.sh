# fused edge head (pooled_fc) on the final tree: all GPU tests + smoke, benches, head A/B at edge batches
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3o}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 --edge 1,8 > gpurun_out/${T}_edge_nohead.txt 2>&1 || exit $?
KVEDGE_FUSE_HEAD=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 --edge 1,8 > gpurun_out/${T}_edge_head.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || exit $?
for f in bench edge_head edge_nohead yolo; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${T}_$f.txt) $(grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_$f.txt)"; done
