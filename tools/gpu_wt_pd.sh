set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for pd in 1 2 3; do
  LFK_BMM_WTPD=$pd timeout -k 10 120 python3 tools/bmm_timeline.py --shapes gate_up_sw --reps 20 2>/dev/null | sed "s/^/pd$pd /" || exit 1
done
for pd in 1 3; do
  LFK_BMM_WTPD=$pd timeout -k 10 200 python3 tools/batch_bench.py --batches 6 --steps 64 2>/dev/null | sed "s/^/pd$pd /" || exit 1
done
