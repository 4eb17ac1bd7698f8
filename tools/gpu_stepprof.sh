# B=6 batch-step kernel stats (no PMC) + the headline bench, one GPU call.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-cur}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof_$tag -o bstep --output-format csv -- \
  python3 tools/batch_bench.py --batches 6 --steps 32 > gpurun_out/bprof_$tag.log 2>&1 || { tail -20 gpurun_out/bprof_$tag.log; exit 1; }
timeout -k 10 200 python3 tools/batch_bench.py --batches 1,6,8 --steps 64 > gpurun_out/bstep_$tag.json 2>gpurun_out/bstep_$tag.err || { tail -20 gpurun_out/bstep_$tag.err; exit 1; }
cat gpurun_out/bstep_$tag.json
if [ "${2:-bench}" = bench ]; then
  timeout -k 10 400 python3 bench.py --steps 5 --warmup 1 > gpurun_out/bench_$tag.json 2>gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
  cat gpurun_out/bench_$tag.json
fi
