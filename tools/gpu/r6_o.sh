# same-box A/B: split-K tile range read from the library (new) vs the pre-fix derived range
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export KVEDGE_AB_OLD_SPLITK=1; else unset KVEDGE_AB_OLD_SPLITK; fi
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6o_${arm}_$i.txt 2>>gpurun_out/r6o.err || exit 1
    echo "$arm $i $(python tools/bench_line.py gpurun_out/r6o_${arm}_$i.txt)"
  done
done
