set -o pipefail
mkdir -p gpurun_out
true
true
for r in 1 2; do timeout -k 10 120 python tools/bmm_bench.py --rows 6 > gpurun_out/q6_mb_new.json 2>/dev/null || exit 1
timeout -k 10 120 python ab_old/tools/bmm_bench.py --rows 6 > gpurun_out/q6_mb_old.json 2>/dev/null || exit 1
echo "mb new $(cat gpurun_out/q6_mb_new.json)"; echo "mb old $(cat gpurun_out/q6_mb_old.json)"; done
bash tools/gpu_ab_old.sh
