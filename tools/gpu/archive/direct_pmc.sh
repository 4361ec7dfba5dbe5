set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python tools/direct_probe.py > gpurun_out/dprobe.log 2>&1 && \
timeout -k 10 120 python tools/direct_probe.py --tile 1 >> gpurun_out/dprobe.log 2>&1 && \
timeout -k 10 120 python tools/direct_probe.py --shape 256,160,160,16,16,3,1 --act 2 >> gpurun_out/dprobe.log 2>&1 && \
bash tools/pmc_cmd.sh gpurun_out/pmc_direct tools/direct_probe.py --reps 3
rc=$?; cat gpurun_out/dprobe.log; exit $rc
