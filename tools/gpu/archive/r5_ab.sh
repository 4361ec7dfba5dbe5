# Round 5 (ab): ResNet-50 stride-2 / stride-1 128-channel 3x3s on the direct family (v10 tile 0,
# 4 waves) vs the implicit-GEMM tiles, isolated at batch 640 with 2 concurrent streams
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5ab}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "direct or every_tile" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 600 python -u tools/tile_probe.py --batch 640 --concurrent 2 --only s2.c2s,s2.c2 --iters 10 > gpurun_out/${T}_tiles.md 2>gpurun_out/${T}_tiles.err || { tail -20 gpurun_out/${T}_tiles.err; exit 1; }
cat gpurun_out/${T}_tiles.md
