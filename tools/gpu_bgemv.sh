#!/bin/bash
# Batched-GEMV session: kernel numerics, batched engine tests, batch_step sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "bmm or bprep" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/bgemv_tests.log 2>&1 || { tail -40 gpurun_out/bgemv_tests.log; exit 1; }
tail -2 gpurun_out/bgemv_tests.log
timeout -k 10 400 python -u -m pytest tests/test_batch_gpu.py tests/test_batch_serving_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/batch_tests.log 2>&1 || { tail -40 gpurun_out/batch_tests.log; exit 1; }
tail -2 gpurun_out/batch_tests.log
timeout -k 10 300 python -u tools/batch_bench.py > gpurun_out/bb_bgemv.log 2>&1 || { tail -20 gpurun_out/bb_bgemv.log; exit 1; }
tail -1 gpurun_out/bb_bgemv.log
if [ "${PROF:-0}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bbprof2 -o bb --output-format csv -- \
    python3 tools/batch_bench.py --batches 8 --steps 16 > gpurun_out/bbprof2.log 2>&1 || exit 1
fi
