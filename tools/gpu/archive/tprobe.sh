set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python tools/tile_probe.py --batch 640 --iters 10 --only ${ONLY:-s3.c3,s3.c1,s3.c2,s2.c2,s2.c3,s4.c3} > gpurun_out/tile_probe.md 2>&1
rc=$?; cat gpurun_out/tile_probe.md; exit $rc
