# Round 6 (f): (1) y_sub with the division-free pixel walk: kernel test + in-graph tables
# KVEDGE_YSUB=1 vs 0; (2) KV_GLDS_IL (fragment reads of k-step ks+1 interleaved between the
# MFMAs of ks) as _C_il.so vs _C.so: tile probe on the GEMM layers, then the headline A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6f}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "ysub" > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 1; }
tail -1 gpurun_out/${T}_pytest.txt
for ys in 1 0; do
  d=gpurun_out/${T}_gl_$ys
  KVEDGE_YSUB=$ys timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o gl -- \
    python3 tools/graph_layers.py run --labels ${d}_labels.json --reps 10 > ${d}.log 2>&1 || { tail -20 ${d}.log; exit 1; }
  python3 tools/graph_layers.py summarize $d --labels ${d}_labels.json --reps 10 > ${d}.md 2>&1 || { tail -20 ${d}.md; exit 1; }
  rm -rf $d
  head -4 ${d}.md | tail -2
  grep -E "^\| (7|9|16|18) \|" ${d}.md | cut -d'|' -f2,3,6,9
done
for lib in _C.so _C_il.so; do
  KVEDGE_LIB=$lib timeout -k 10 300 python -u tools/tile_probe.py --batch 640 --only s2.c2,s3.c2,s4.c2,s3.c2s,s4.c2s,s3.c1,s4.c1,s3.c3-nores --tiles 29,80,83 > gpurun_out/${T}_tiles_$lib.md 2>&1 || { tail -20 gpurun_out/${T}_tiles_$lib.md; exit 1; }
  echo "== $lib"; grep "^| s" gpurun_out/${T}_tiles_$lib.md
done
for r in 1 2; do
for lib in _C.so _C_il.so; do
  KVEDGE_LIB=$lib KVEDGE_BENCH_YOLO=0 KVEDGE_EDGE= timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 > gpurun_out/${T}_b_${lib}_$r.txt 2>gpurun_out/${T}_b.err || { tail -20 gpurun_out/${T}_b.err; exit 1; }
  echo "$lib $(python tools/bench_line.py gpurun_out/${T}_b_${lib}_$r.txt)"
done
done
