#!/bin/bash
# GEMV structure experiments: block size x (rows, passes), with the debug
# variants (dbg1: no x prologue, dbg2: prologue + first loads, dbg3: weights after prologue)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for blk in 256 1024; do
  for cfg in "" "4,1" "2,2" "1,4"; do
    echo "blk=$blk cfg=[$cfg]"
    LFK_GEMV_BLOCK=$blk LFK_GEMV_CFG="$cfg" timeout -k 10 120 python tools/gemv_bench.py --reps 30 --debug --only q4k || exit $?
  done
done
