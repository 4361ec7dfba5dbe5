#!/bin/bash
# A/B two builds of the native library on ONE box (box-to-box spread is larger than most
# single-kernel changes): tools/ab_lib.sh MODEL BATCH libA libB  (kvedge_amd/_C_<lib>.so)
# alternates A B A B, one rocprofv3 forward table per run, under gpurun_out/ab/.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
model=$1 batch=$2; shift 2
mkdir -p gpurun_out/ab
cp kvedge_amd/_C.so /tmp/_C_keep.so
for i in 1 2; do
  for lib in "$@"; do
    cp "kvedge_amd/_C_$lib.so" kvedge_amd/_C.so
    d=gpurun_out/ab/${lib}_$i
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d -o t -- \
      python3 tools/profile_forward.py --model $model --batch $batch > $d.log 2>&1 || { cp /tmp/_C_keep.so kvedge_amd/_C.so; exit 3; }
    python tools/profile_forward.py --summarize $d/t_kernel_trace.csv > $d.md
    rm -rf $d
    echo "$lib run $i: $(head -1 $d.md)"
  done
done
cp /tmp/_C_keep.so kvedge_amd/_C.so
