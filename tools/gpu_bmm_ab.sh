# bmm A/B session: kernel numerics, batched-engine tests, batch-step sweeps under the
# tuning switches (env assignments given as arguments, "-" = defaults), then the headline
# bench. Every GPU step has its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_batch_gpu.py -x -q -k "bmm or bprep or batch" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -3 gpurun_out/ab_tests.log
i=0
for v in "$@"; do
  i=$((i + 1))
  if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 200 python tools/batch_bench.py > gpurun_out/ab_$i.json 2>> gpurun_out/ab.err || exit 1
  echo "$v $(cat gpurun_out/ab_$i.json)"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || exit 1
cat gpurun_out/ab_bench.json
