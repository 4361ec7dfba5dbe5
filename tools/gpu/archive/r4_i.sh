# Round 4 (i): direct-family fragment ring depth 8 (DMA forms): numerics + per-layer probe
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4i}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "direct or canary or pair" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for sp in "192,80,80,64,128,3,1 silu" "192,80,80,64,16,3,1 silu" "640,56,56,64,64,3,1 relu" "192,80,80,32,32,3,1 silu" "192,40,40,64,64,3,1 silu" "192,160,160,32,64,3,2 silu" "640,28,28,128,128,3,1 relu"; do set -- $sp
  echo "## $1 $2" >> gpurun_out/${T}_probe.txt; timeout -k 10 120 python3 tools/conv_probe.py --shape $1 --act $2 --tiles 54,55,105,107 --iters 20 >> gpurun_out/${T}_probe.txt 2>&1 || { tail -5 gpurun_out/${T}_probe.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/${T}_probe.txt
