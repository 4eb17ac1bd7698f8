# Same-box kernel-level A/B: rocprofv3 kernel stats of the B = 6 batch step for the tree's build,
# the staged older build (ab_old/) and env variants of the tree's build.
# usage: bash tools/gpu_abprof.sh "LABEL=ENV ..." ...   (always runs "new" and "old")
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <label> <batch_bench.py path> [env...]
  local lab=$1 bb=$2; shift 2
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$lab -o bstep --output-format csv -- \
    python3 $bb --batches 6 --steps 32 > gpurun_out/abp_$lab.log 2>&1 || { tail -20 gpurun_out/abp_$lab.log; exit 1; }
  python3 tools/step_kernels.py gpurun_out/abp_$lab/bstep_kernel_trace.csv > gpurun_out/abp_$lab.txt
  echo "== $lab"; cat gpurun_out/abp_$lab.txt
}
run new tools/batch_bench.py
run old ab_old/tools/batch_bench.py
for v in "$@"; do
  lab=${v%%=*}; envs=${v#*=}
  run "$lab" tools/batch_bench.py $envs
done
