#!/bin/bash
# Kernel traces of the serving steps for tools/step_timeline.py: the B=6 batch step and the
# single-row graph decode (batch_bench --batches 1 runs batch_step over one row = the
# single-row GEMV graph of that slot).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=${1:-6}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/st_b$B -o st --output-format csv -- \
  python3 tools/batch_bench.py --batches $B --steps 24 --slots 8 > gpurun_out/st_b$B.log 2>&1 || { tail -20 gpurun_out/st_b$B.log; exit 1; }
f=$(find gpurun_out/st_b$B -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$f" --steps 16 --json gpurun_out/st_b$B.json
