# Round 5 (af): ResNet-50 b1280 headline with 2 vs 4 stream slices (640 vs 320 images per slice)
# on this round's kernels, alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5af}
for r in 1 2; do
for s in 2 4; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --streams $s --edge '' --yolo 0 > gpurun_out/${T}_s${s}_$r.txt 2>gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
  echo "streams=$s $(python tools/bench_line.py gpurun_out/${T}_s${s}_$r.txt)"
done
done
