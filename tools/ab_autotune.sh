cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
 for r in 0 20; do
  for m in resnet50 yolov8n; do
   KVEDGE_AUTOTUNE_REFINE_ITERS=$r timeout -k 10 120 python bench.py --model $m --steps 30 --warmup 5 > gpurun_out/ab_${m}_r${r}_$i.log 2>&1 || exit $?
   echo "$m refine=$r run=$i $(grep -o '"value": [0-9.]*' gpurun_out/ab_${m}_r${r}_$i.log)"
  done
 done
done
