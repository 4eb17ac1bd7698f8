# bmm A/B session: kernel numerics, batched-engine tests, batch-step sweeps under the
# tuning switches, then the headline bench. Every GPU step has its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_batch_gpu.py -x -q -k "bmm or bprep or batch" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -3 gpurun_out/ab_tests.log
timeout -k 10 200 python tools/batch_bench.py > gpurun_out/ab_default.json 2> gpurun_out/ab_default.err || exit 1
cat gpurun_out/ab_default.json
LFK_BMM_SIDE=0 timeout -k 10 200 python tools/batch_bench.py > gpurun_out/ab_noside.json 2>> gpurun_out/ab_default.err || exit 1
cat gpurun_out/ab_noside.json
LFK_BMM_NW1=4 timeout -k 10 200 python tools/batch_bench.py > gpurun_out/ab_nw4.json 2>> gpurun_out/ab_default.err || exit 1
cat gpurun_out/ab_nw4.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err || exit 1
cat gpurun_out/ab_bench.json
