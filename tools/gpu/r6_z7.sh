# Round 6 (z7): headline batch / stream-slice sweep on one box with the round-6 kernels
# (640-image slices x 2 / 3 / 4 streams, 320 x 4, 960 x 2), alternated with the default
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z7}
for cfg in "1280 2" "1920 3" "2560 4" "1280 4" "1920 2" "1280 2"; do
  set -- $cfg
  KVEDGE_BENCH_YOLO=0 KVEDGE_EDGE= timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --batch $1 --streams $2 > gpurun_out/${T}_b$1_s$2.txt 2>>gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
  echo "b$1 s$2: $(python tools/bench_line.py gpurun_out/${T}_b$1_s$2.txt)"
done
