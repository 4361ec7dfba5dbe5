# 128x160 DE tiles (N = 144 Detect stems): tests, benches, YOLO op roofline, ResNet b640 roofline
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3l}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || exit $?
for f in bench yolo; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${T}_$f.txt) $(grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_$f.txt)"; done
timeout -k 10 400 python -u tools/op_roofline.py --model yolov8n --batch 192 --streams 2 \
  > gpurun_out/${T}_yolo_roofline_b192.md 2> gpurun_out/${T}_yolo_roofline.err || exit $?
grep "Forward\|Largest" gpurun_out/${T}_yolo_roofline_b192.md
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_fwd -o fwd -- \
  python3 tools/profile_forward.py --batch 640 > gpurun_out/${T}_fwd640.log 2>&1 && \
python tools/roofline_table.py gpurun_out/${T}_fwd/fwd_kernel_trace.csv --batch 640 > gpurun_out/${T}_roofline_b640.md
rc=$?
rm -rf gpurun_out/${T}_fwd
tail -1 gpurun_out/${T}_roofline_b640.md
exit $rc
