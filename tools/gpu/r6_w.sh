# Round 6 (w): v14 phase-budget ablation (tools/pp_abl.py, KVEDGE_PP_ABL instantiations)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6w}
for L in s3.c2 s4.c2 s3.c1; do
  for A in 0 1 2 4 6 8 16 22; do
    KVEDGE_PP_ABL=$A timeout -k 10 120 python -u tools/pp_abl.py --layer $L --batch 640 > gpurun_out/${T}_${L}_$A.txt 2>&1 || { tail -20 gpurun_out/${T}_${L}_$A.txt; exit 1; }
    grep "per launch" gpurun_out/${T}_${L}_$A.txt
  done
done
