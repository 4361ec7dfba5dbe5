# Round 5 (ag): phase-pipelined slices (KVEDGE_PHASE=1: slice 1 half a network behind slice 0)
# vs the lock-step slices: engine stream tests, then the b1280 headline alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ag}
timeout -k 10 600 python -u -m pytest tests/test_engine_streams_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2; do
for ph in 1 0; do
  KVEDGE_PHASE=$ph timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge '' --yolo 0 > gpurun_out/${T}_p${ph}_$r.txt 2>gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
  echo "phase=$ph $(python tools/bench_line.py gpurun_out/${T}_p${ph}_$r.txt)"
done
done
for k in 5 7; do
  KVEDGE_PHASE=1 KVEDGE_PHASE_SPLIT=$k timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge '' --yolo 0 > gpurun_out/${T}_k${k}.txt 2>gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
  echo "phase=1 split=$k $(python tools/bench_line.py gpurun_out/${T}_k${k}.txt)"
done
