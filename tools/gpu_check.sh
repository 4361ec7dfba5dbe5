#!/bin/bash
# One gpurun session: numerics tests, smoke, headline bench, torch yard-stick, rocprof.
# Every GPU step has its own timeout; a crash/timeout/abort ends the script (no retries).
# Usage: tools/gpu_check.sh [steps...]   steps: test smoke bench base prof sweep
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS="${*:-test smoke bench base prof}"

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  local t0=$SECONDS
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc wall=$((SECONDS - t0))s" | tee -a $OUT/steps.log
  tail -n 5 "$OUT/$name.log"
  # 0 ok, 1 = test failures (not a GPU fault); anything else = stop touching the GPU
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping after $name (rc=$rc)" | tee -a $OUT/steps.log
    exit $rc
  fi
}

for s in $STEPS; do
  case $s in
    test)  run pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py --steps 30 --warmup 5 --json-out $OUT/bench.json ;;
    yolo)  run bench_yolo 400 python bench.py --model yolov8n --steps 20 --warmup 3 --json-out $OUT/bench_yolo.json ;;
    base)  run torch_base 400 python tools/torch_baseline.py --graph --batch 256 ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 2 ;;
    sweep) run sweep 600 python tools/batch_sweep.py ;;
    pmc)   run pmc 1000 bash tools/prof_layers.sh 256 ;;
    fwd)   run fwdprof 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/fwd -o fwd -- python3 tools/profile_forward.py --batch 640 &&
           python tools/profile_forward.py --summarize $OUT/fwd/fwd_kernel_trace.csv > $OUT/fwd_summary.md ;;
    fwdyolo) run fwdyolo 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/fwdy -o fwdy -- python3 tools/profile_forward.py --model yolov8n --batch 256 &&
           python tools/profile_forward.py --summarize $OUT/fwdy/fwdy_kernel_trace.csv > $OUT/fwd_yolo_summary.md ;;
    rccl)  run rccl 300 ./kvedge_amd/bin/kv_rccl_bench 1024 268435456 10 bf16 ;;
    layers64) run layers64 600 python tools/layer_bench.py --batch 64 --out $OUT/layer_bench_b64.md ;;
    layers) run layers 600 python tools/layer_bench.py ;;
  esac
done
echo "=== all done" | tee -a $OUT/steps.log
