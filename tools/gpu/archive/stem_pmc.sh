set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/pmc_cmd.sh gpurun_out/pmc_stem2 tools/stem_probe.py --reps 3 > gpurun_out/pmc_stem2.log 2>&1
