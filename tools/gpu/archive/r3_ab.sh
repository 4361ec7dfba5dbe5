# Round 3, session 2: split-K fixup without fences, in-kernel counter bump, softmax rows
# (tests); stem prefetch depth A/B (kvedge_amd/_C_ab.so = this tree with the one-band stems)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3f}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "splitk or synth or softmax" > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
for i in 1 2; do
  timeout -k 10 200 python -u tools/stem_ab.py >> gpurun_out/${T}_stem.txt 2>&1 || exit $?
  KVEDGE_LIB=_C_ab.so timeout -k 10 200 python -u tools/stem_ab.py >> gpurun_out/${T}_stem.txt 2>&1 || exit $?
done
cat gpurun_out/${T}_stem.txt | grep '^{'
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.txt 2>&1 || exit $?
KVEDGE_LIB=_C_ab.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_bench_ab.txt 2>&1 || exit $?
KVEDGE_SK_FINALIZE=1 timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --batch 64 > gpurun_out/${T}_edge_fin.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo.txt 2>&1 || exit $?
KVEDGE_LIB=_C_ab.so timeout -k 10 400 python -u bench.py --model yolov8n --steps 20 --warmup 5 --edge "" > gpurun_out/${T}_yolo_ab.txt 2>&1 || exit $?
for f in bench bench_ab edge_fin yolo yolo_ab; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${T}_$f.txt) $(grep -o '"edge": \[[^]]*\]' gpurun_out/${T}_$f.txt)"; done
