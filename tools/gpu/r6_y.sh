# Round 6 (y): v14 staging cache policy -- A / B / both LDS-DMAs non-temporal (KVEDGE_PP_ABL
# 32 / 64 / 96: correct outputs) vs default, alternated, three layers
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6y}
for r in 1 2; do
for L in s3.c2 s4.c2 s3.c1; do
  for A in 0 32 64 96; do
    KVEDGE_PP_ABL=$A timeout -k 10 120 python -u tools/pp_abl.py --layer $L --batch 640 > gpurun_out/${T}_${L}_${A}_$r.txt 2>&1 || { tail -20 gpurun_out/${T}_${L}_${A}_$r.txt; exit 1; }
    grep "per launch" gpurun_out/${T}_${L}_${A}_$r.txt
  done
done
done
