#!/bin/bash
# GEMV (rows-per-item, passes) sweep: one process per LFK_GEMV_CFG value.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "" "4,2" "4,1" "2,4" "2,2" "2,1" "1,4" "1,2"; do
  echo "cfg=[$cfg]"
  LFK_GEMV_CFG="$cfg" timeout -k 10 120 python tools/gemv_bench.py --reps 50 || exit $?
done
