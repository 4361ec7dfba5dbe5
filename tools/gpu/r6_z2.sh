# Round 6 (z2): v15 deep-ring 256 x 256 4-wave tiles (121-123) -- correctness, then eager
# timing against v14 (117) and de:80 on the ResNet layers
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z2}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "121 or 122 or 123 or tile_count" --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 400 python -u tools/tile_probe.py --batch 640 --tiles 80,117,121,122,123 --only s3.c2,s4.c2,s3.c1,s4.c1,s3.c2s,s4.c2s,s4.c3,s3.c3-nores,s2.c2 > gpurun_out/${T}_tiles.md 2>&1 || { tail -20 gpurun_out/${T}_tiles.md; exit 1; }
grep "^|" gpurun_out/${T}_tiles.md
