# Round 4 (n): fused-tail GEMM fragment ring (conv_stream.hip) A/B vs _C_ab.so (previous tail);
# direct tests + strided CIN-128 probe; ResNet v10 on/off; b1 / b64 forward profiles + edge
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4n}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "tail or stream or direct or tile_count" > gpurun_out/${T}_t.txt 2>&1 || { tail -40 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 120 python3 tools/conv_probe.py --shape 640,56,56,128,128,3,2 --act relu --tiles 29,80,82,105 --iters 20 > gpurun_out/${T}_probe.txt 2>&1 || { tail -5 gpurun_out/${T}_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_probe.txt
for r in 1 2; do
  for lib in _C.so _C_ab.so; do
    KVEDGE_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_resnet_${lib}_$r.txt 2>&1 || { tail -5 gpurun_out/${T}_resnet_${lib}_$r.txt; exit 1; }
    echo "$lib $r $(grep -o '"value": [0-9.]*' gpurun_out/${T}_resnet_${lib}_$r.txt | head -1)"
  done
done
KVEDGE_TILE_LIMIT=105 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_resnet_nov10.txt 2>&1 || { tail -5 gpurun_out/${T}_resnet_nov10.txt; exit 1; }
echo "no-v10 $(grep -o '"value": [0-9.]*' gpurun_out/${T}_resnet_nov10.txt | head -1)"
for b in 1 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_b$b -o b$b -- python3 tools/profile_forward.py --batch $b --reps 20 > gpurun_out/${T}_b$b.log 2>&1 || { tail -5 gpurun_out/${T}_b$b.log; exit 1; }
  python3 tools/profile_forward.py --summarize gpurun_out/${T}_b$b/b${b}_kernel_trace.csv --reps 20 > gpurun_out/${T}_b${b}_forward.md 2>&1 || exit 1
  head -8 gpurun_out/${T}_b${b}_forward.md
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/${T}_edge.txt 2>&1 || { tail -5 gpurun_out/${T}_edge.txt; exit 1; }
grep -o '"edge": .*' gpurun_out/${T}_edge.txt | cut -c1-400
