# Round 6 (v): v14 phase anatomy (KV_PP_TRACE build, tools/pp_trace.py) on the layers it runs
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6v}
for L in s3.c2 s4.c2 s3.c1 s3.c2s; do
  KVEDGE_LIB=_C_trace.so timeout -k 10 120 python -u tools/pp_trace.py --layer $L --batch 640 > gpurun_out/${T}_$L.txt 2>&1 || { tail -20 gpurun_out/${T}_$L.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_$L.txt
done
KVEDGE_LIB=_C_trace.so timeout -k 10 120 python -u tools/pp_trace.py --layer s2.c2 --batch 640 --tile 118 > gpurun_out/${T}_s2.c2_118.txt 2>&1 || { tail -20 gpurun_out/${T}_s2.c2_118.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_s2.c2_118.txt
