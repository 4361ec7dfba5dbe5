# Round 6 (z10): v14 ablation, A vs B staging: which DMA stream costs, and with / without the
# fragment reads (KVEDGE_PP_ABL 32 no B DMA, 64 no A DMA, 34 / 66 the same without reads)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6z10}
for L in s3.c2 s4.c2 s3.c1; do
  for A in 0 32 64 4 2 34 66 6; do
    KVEDGE_PP_ABL=$A timeout -k 10 120 python -u tools/pp_abl.py --layer $L --batch 640 > gpurun_out/${T}_${L}_$A.txt 2>&1 || { tail -20 gpurun_out/${T}_${L}_$A.txt; exit 1; }
    grep "per launch" gpurun_out/${T}_${L}_$A.txt
  done
done
