# Same-box A/B of env-selected kernel variants on the batched step (+ optional tests/profile).
#   bash tools/gpu_ab_env.sh <tag> "<envA>" "<envB>" [tests] [prof]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; A=$2; Bv=$3
if [ "${4:-}" = tests ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_batch_gpu.py tests/test_engine_gpu.py > gpurun_out/tests_$tag.txt 2>&1 || { tail -30 gpurun_out/tests_$tag.txt; exit 1; }
  tail -3 gpurun_out/tests_$tag.txt
fi
for i in 1 2; do
  for v in A B; do
    e=$A; [ $v = B ] && e=$Bv
    env $e timeout -k 10 200 python3 tools/batch_bench.py --batches 1,6,8 --steps 64 > gpurun_out/ab_${tag}_$v$i.json 2>/dev/null || exit 1
    echo "$v$i [$e] $(cat gpurun_out/ab_${tag}_$v$i.json)"
  done
done
if [ "${5:-}" = prof ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof_$tag -o bstep --output-format csv -- \
    python3 tools/batch_bench.py --batches 6 --steps 32 > gpurun_out/bprof_$tag.log 2>&1 || { tail -20 gpurun_out/bprof_$tag.log; exit 1; }
fi
