# Batch-step profile: kernel trace + stats at B=6, then one PMC pass (own run, no tracing).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o bstep --output-format csv -- \
  python3 tools/batch_bench.py --batches 6 --steps 32 > gpurun_out/bprof.log 2>&1 || { tail -20 gpurun_out/bprof.log; exit 1; }
find gpurun_out/bprof -name "*kernel_stats.csv" | head -3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  -d gpurun_out/bpmc -o pmc --output-format csv -- python3 tools/batch_bench.py --batches 6 --steps 4 > gpurun_out/bpmc.log 2>&1 || { tail -20 gpurun_out/bpmc.log; exit 1; }
find gpurun_out/bpmc -name "*.csv" | head -5
