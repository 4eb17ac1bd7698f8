#!/bin/bash
# Split-K launch-shape sweep of the batched projections (LFK_BMM_XKB: staged-x budget -> K part
# length, LFK_BMM_GRID: blocks per CU), one process per setting (the knobs are read once).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for xkb in 32 16 8; do
  for grid in 4 2; do
    echo "=== xkb=$xkb grid=$grid"
    LFK_BMM_XKB=$xkb LFK_BMM_GRID=$grid timeout -k 10 120 python tools/bmm_timeline.py --rows 6 --shapes wq,down,down6,wk --reps 6 2>/dev/null | cut -c1-200 || exit 1
  done
done
