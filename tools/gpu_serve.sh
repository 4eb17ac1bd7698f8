#!/bin/bash
# Continuous-batching GPU session: batched numerics + serving tests, then the default
# (6 clients, continuous batch) and serial (1 client, max_batch 1) /response benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_batch_gpu.py tests/test_batch_serving_gpu.py -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/serve_tests.log 2>&1 || { tail -40 gpurun_out/serve_tests.log; exit 1; }
tail -3 gpurun_out/serve_tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 > gpurun_out/bench_c6.log 2>gpurun_out/bench_c6.err || { tail -20 gpurun_out/bench_c6.err; exit 1; }
tail -1 gpurun_out/bench_c6.log
if [ "${SERIAL:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py --steps 10 --warmup 1 --clients 1 --max-batch 1 > gpurun_out/bench_c1.log 2>gpurun_out/bench_c1.err || { tail -20 gpurun_out/bench_c1.err; exit 1; }
  tail -1 gpurun_out/bench_c1.log
fi
