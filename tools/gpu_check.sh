#!/bin/bash
# One gpurun call's worth of checks on a fresh MI355X box, every GPU step under its own
# time limit and chained with && (a fault, abort or timeout ends the call there).
#   bash tools/gpu_check.sh TAG [STEPS...]
# STEPS (default: tests smoke bench yolo): tests | kernels | smoke | bench | yolo | edge
# Output: gpurun_out/TAG_<step>.txt
set -o pipefail
tag=${1:?tag}; shift
steps=${*:-tests smoke bench yolo}
mkdir -p gpurun_out
for s in $steps; do
  out=gpurun_out/${tag}_${s}.txt
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
             --timeout-method thread > "$out" 2>&1 ;;
    kernels) timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
             --timeout-method thread > "$out" 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out" 2>&1 ;;
    bench) timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > "$out" 2>&1 ;;
    yolo) timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" \
             > "$out" 2>&1 ;;
    edge) timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 > "$out" 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "step $s rc=$rc"
  tail -3 "$out"
  [ $rc -eq 0 ] || exit $rc
done
