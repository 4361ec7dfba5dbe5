# Round 4 (b): seam tile forms (4-wave 2-per-CU, 16-KB stages) and v10 persistent tiles, same box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4b}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "seam or pde" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u tools/seam_probe.py --batch 640 > gpurun_out/${T}_seam_probe.md 2>&1 || { cat gpurun_out/${T}_seam_probe.md; exit 1; }
cat gpurun_out/${T}_seam_probe.md
timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --iters 10 --only s3.c2,s4.c2,s3.c1,s3.c2s,s4.c2s,s2.c2,s4.c1 \
  --tiles 78,79,80,81,86,87,88 > gpurun_out/${T}_tiles.md 2>&1 || exit $?
cat gpurun_out/${T}_tiles.md
timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --iters 10 --concurrent 2 --only s3.c2,s4.c2,s3.c1,s4.c1 \
  --tiles 78,79,80,81,86,87,88 > gpurun_out/${T}_tiles_c2.md 2>&1 || exit $?
cat gpurun_out/${T}_tiles_c2.md
