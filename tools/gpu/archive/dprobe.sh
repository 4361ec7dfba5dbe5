set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/dprobe.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py -k "direct or stem or yolo or resnet" > gpurun_out/dtest.log 2>&1 && \
for s in 640,56,56,64,64,3,1:1 256,160,160,16,16,3,1:2 256,80,80,32,32,3,1:2 256,40,40,64,64,3,1:2; do
  timeout -k 10 120 python tools/direct_probe.py --shape ${s%:*} --act ${s#*:} >> gpurun_out/dprobe.log 2>&1 || exit $?
done
rc=$?; tail -2 gpurun_out/dtest.log; grep tile gpurun_out/dprobe.log; exit $rc
timeout -k 10 120 python tools/stem_probe.py >> gpurun_out/dprobe.log 2>&1
