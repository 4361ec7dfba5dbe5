set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $P tests/test_models_gpu.py -k "stem12 or stem_pool_frames" > gpurun_out/pytest_stem12.log 2>&1
rc=$?; tail -n 15 gpurun_out/pytest_stem12.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stem_probe.py --batch 640 > gpurun_out/stem_probe.txt 2>&1 && cat gpurun_out/stem_probe.txt && \
timeout -k 10 400 bash tools/pmc_layer.sh s3.c2 30 gpurun_out/pmc30 && \
timeout -k 10 400 bash tools/pmc_layer.sh s3.c2 68 gpurun_out/pmc68 && \
cat gpurun_out/pmc30/summary.txt gpurun_out/pmc68/summary.txt
