# Same-box: this tree (default), this tree with the new bmm paths off (env), and the build
# staged in ab_old/, alternating; then the attention timeline and the headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OFF="LFK_BMM_WT=0 LFK_BMM_WTK=0 LFK_BMM_QKV2=0"
for r in 1 2; do
  timeout -k 10 200 python3 tools/batch_bench.py --batches 1,6,8 > gpurun_out/ab3_new_$r.json 2>/dev/null || exit 1
  echo "new $(cat gpurun_out/ab3_new_$r.json)"
  env $OFF timeout -k 10 200 python3 tools/batch_bench.py --batches 1,6,8 > gpurun_out/ab3_off_$r.json 2>/dev/null || exit 1
  echo "off $(cat gpurun_out/ab3_off_$r.json)"
  timeout -k 10 200 python3 ab_old/tools/batch_bench.py --batches 1,6,8 > gpurun_out/ab3_old_$r.json 2>/dev/null || exit 1
  echo "old $(cat gpurun_out/ab3_old_$r.json)"
done
timeout -k 10 120 python3 tools/attn_timeline.py --rows 6 --L 700 > gpurun_out/attn_tl.txt 2>/dev/null || exit 1
cat gpurun_out/attn_tl.txt
timeout -k 10 400 python3 bench.py --steps 5 --warmup 1 > gpurun_out/bench_ab3.json 2>gpurun_out/bench_ab3.err || { tail -5 gpurun_out/bench_ab3.err; exit 1; }
cat gpurun_out/bench_ab3.json
