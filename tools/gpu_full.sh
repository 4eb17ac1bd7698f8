#!/bin/bash
# Round-end style GPU session: every GPU test, the smoke entry point, the default bench
# (6 clients, continuous batch) and the serial bench, plus a kernel profile of batch steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 > gpurun_out/bench_c6.log 2>gpurun_out/bench_c6.err || { tail -20 gpurun_out/bench_c6.err; exit 1; }
tail -1 gpurun_out/bench_c6.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 1 --clients 1 --max-batch 1 > gpurun_out/bench_c1.log 2>gpurun_out/bench_c1.err || { tail -20 gpurun_out/bench_c1.err; exit 1; }
tail -1 gpurun_out/bench_c1.log
