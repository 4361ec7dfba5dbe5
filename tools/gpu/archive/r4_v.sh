# Round 4 (v): direct-epilogue stores non-temporal (diag 16) vs default, same box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4v}
for sp in "192,80,80,64,128,3,1 silu" "640,56,56,64,64,3,1 relu" "192,40,40,64,64,3,1 silu"; do set -- $sp
  for d in 0 16 0 16; do
    echo "## $1 $2 diag=$d" >> gpurun_out/${T}_diag.txt
    KVEDGE_DIRECT_DIAG=$d timeout -k 10 120 python3 tools/conv_probe.py --shape $1 --act $2 --tiles 105,107 --iters 20 >> gpurun_out/${T}_diag.txt 2>&1 || { tail -5 gpurun_out/${T}_diag.txt; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/${T}_diag.txt
