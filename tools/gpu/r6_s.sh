# Round 6 (s): stem12 with the commit normalisation on whole dwords (v_cvt_f32_ubyteN, paired
# bf16 packs, b-term zeroed instead of per-element selects), band-invariant load geometry and
# the bias as the first MFMA's C operand -- GPU tests, stem probe and headline/edge A/B against
# the previous stem12 (kvedge_amd/_C_old.so), alternated on one box
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6s}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "stem or resnet" --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for r in 1 2; do
  for lib in _C.so _C_old.so; do
    KVEDGE_LIB=$lib timeout -k 10 300 python -u tools/stem_probe.py --batch 640 > gpurun_out/${T}_stem_${lib}_$r.txt 2>&1 || { tail -20 gpurun_out/${T}_stem_${lib}_$r.txt; exit 1; }
    echo "$lib $r: $(grep stem12 gpurun_out/${T}_stem_${lib}_$r.txt)"
  done
done
for r in 1 2; do
  for lib in _C.so _C_old.so; do
    KVEDGE_LIB=$lib KVEDGE_BENCH_YOLO=0 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_b_${lib}_$r.txt 2>>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
    echo "$lib $r: $(python tools/bench_line.py gpurun_out/${T}_b_${lib}_$r.txt)"
  done
done
