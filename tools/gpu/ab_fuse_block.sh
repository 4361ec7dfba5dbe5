# A/B under the two-stream bench: fused stage-1 bottleneck body (conv_block.hip) off / on
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for fb in 0 1; do
KVEDGE_FUSE_BLOCK=$fb timeout -k 10 150 python bench.py --steps 30 --warmup 5 2>/dev/null | grep metric | sed "s/^/{\"fuse_block\": $fb, \"r\": /; s/$/}/" >> gpurun_out/ab_fuse_block.jsonl || exit $?
done; done
