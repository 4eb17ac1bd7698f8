set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_batch_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/batch.log 2>&1; rc=$?; tail -30 gpurun_out/batch.log; exit $rc
