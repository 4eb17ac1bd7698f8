set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "state or facade" > gpurun_out/samp.log 2>&1; rc=$?; tail -15 gpurun_out/samp.log; exit $rc
