# DP rehearsal of the driver's N>1 bench on a one-GPU box: 2 ranks, both on GPU 0.
set -o pipefail
mkdir -p gpurun_out
LFK_BENCH_DEVICE=0 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/dp2.log 2>&1
rc=$?; grep '^{"metric"' gpurun_out/dp2.log; tail -5 gpurun_out/dp2.log; exit $rc
