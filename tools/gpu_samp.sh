set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "sampler or facade" > gpurun_out/samp.log 2>&1; rc=$?; tail -15 gpurun_out/samp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench2.log 2>&1; rc=$?; grep '^{"metric"' gpurun_out/bench2.log; exit $rc
