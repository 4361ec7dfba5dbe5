# Round 6 (g): v14 8-phase ping-pong tile (conv_pp.hip, tile 117): correctness first, then
# the tile probe against de:80 at b640, then the headline (the autotuner now sees tile 117)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6g}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_pp or (every_tile and 117) or (dual and 117) or (skinny and 117) or tile_count" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --only s2.c2,s3.c2,s4.c2,s2.c2s,s3.c2s,s4.c2s,s3.c1,s4.c1,s3.c3-nores,s4.c3,s2.c1 --tiles 80,117 > gpurun_out/${T}_tiles.md 2>&1 || { tail -20 gpurun_out/${T}_tiles.md; exit 1; }
grep "^|" gpurun_out/${T}_tiles.md
timeout -k 10 400 python -u tools/tile_probe.py --batch 640 --concurrent 2 --only s3.c2,s4.c2,s3.c1,s4.c1,s3.c2s --tiles 80,117 > gpurun_out/${T}_tiles_c2.md 2>&1 || { tail -20 gpurun_out/${T}_tiles_c2.md; exit 1; }
grep "^|" gpurun_out/${T}_tiles_c2.md
