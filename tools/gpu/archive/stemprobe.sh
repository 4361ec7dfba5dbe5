set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python tools/stem_probe.py --reps 20 > gpurun_out/stem_probe.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/stemprof -o sp -- python3 tools/stem_probe.py --reps 5 > gpurun_out/stem_prof.log 2>&1
rc=$?; cat gpurun_out/stem_probe.log; exit $rc
