# Round 5 (s): fused C2f, one block per wave + hoisted fragment reads: tests, probe, YOLO bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r5s}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "c2f16" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 300 python -u tools/c2f_probe.py --batch 256 --strips 40,20,8 --diags 0,1,6,7 > gpurun_out/${T}_probe.txt 2>&1 || { tail -20 gpurun_out/${T}_probe.txt; exit 1; }
cat gpurun_out/${T}_probe.txt
timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 5 > gpurun_out/${T}_yolo.txt 2>gpurun_out/${T}_yolo.err || { tail -20 gpurun_out/${T}_yolo.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_yolo.txt').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
