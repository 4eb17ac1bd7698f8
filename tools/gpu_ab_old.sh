# Same-box A/B of the batched step: the tree's build against an older build staged in
# ab_old/ (package + batch_bench.py copied from a git worktree of the older commit),
# alternating runs so box drift hits both.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python tools/batch_bench.py --batches 1,6,8 > gpurun_out/abo_new_$r.json 2>> gpurun_out/abo.err || exit 1
  echo "new $(cat gpurun_out/abo_new_$r.json)"
  timeout -k 10 200 python ab_old/tools/batch_bench.py --batches 1,6,8 > gpurun_out/abo_old_$r.json 2>> gpurun_out/abo.err || exit 1
  echo "old $(cat gpurun_out/abo_old_$r.json)"
done
