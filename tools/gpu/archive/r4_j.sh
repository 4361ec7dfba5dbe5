# Round 4 (j): where the direct-epilogue band time goes: KVEDGE_DIRECT_DIAG drops stores (1),
# the next-band prefetch (2), the MFMAs (4) -- timing only, outputs wrong
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4j}
for sp in "192,80,80,64,128,3,1 silu" "640,56,56,64,64,3,1 relu"; do set -- $sp
  for d in 0 1 2 3 4 5 6 7; do
    echo "## $1 $2 diag=$d" >> gpurun_out/${T}_diag.txt
    KVEDGE_DIRECT_DIAG=$d timeout -k 10 120 python3 tools/conv_probe.py --shape $1 --act $2 --tiles 105 --iters 20 >> gpurun_out/${T}_diag.txt 2>&1 || { tail -5 gpurun_out/${T}_diag.txt; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/${T}_diag.txt
