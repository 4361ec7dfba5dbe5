# Round 4 (final 2): all GPU tests + smoke on the tree with the SPPF keys, then a ResNet-50
# batch sweep on one box (alternating order) to re-check the bench default
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r4s}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t.txt 2>&1 || { tail -30 gpurun_out/${T}_t.txt; exit 1; }
tail -1 gpurun_out/${T}_t.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.txt
for b in 1280 1536 1024 1280 1536 1024; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --edge "" --batch $b > gpurun_out/${T}_b$b.txt 2>&1 || { tail -5 gpurun_out/${T}_b$b.txt; exit 1; }
  echo "batch $b: $(grep -o '"value": [0-9.]*' gpurun_out/${T}_b$b.txt | head -1)" | tee -a gpurun_out/${T}_sweep.txt
done
