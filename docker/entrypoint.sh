#!/bin/bash
# Container entry: one rank per GPU.
#   GPUS_PER_POD=1 (default)  -> gunicorn -w $WORKERS_PER_GPU -k uvicorn.workers.UvicornWorker api:app
#                                (reference CMD with WORKERS_PER_GPU=1, the default; each extra worker is
#                                one more independent replica - its own engine, queue and KV cache - on
#                                the same 288 GB GPU: 2 workers measured 1.35x the decode tokens/s of one)
#   GPUS_PER_POD=N, N>1       -> torchrun, N ranks, SPLIT_MODE=row (tensor parallel over RCCL/xGMI);
#                                rank 0 serves HTTP, the others follow.
set -euo pipefail
N=${GPUS_PER_POD:-1}
PORT=${PORT:-8000}
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$N" -le 1 ]; then
  exec gunicorn -w "${WORKERS_PER_GPU:-1}" -k uvicorn.workers.UvicornWorker api:app --bind "0.0.0.0:${PORT}" --timeout 0
fi
export SPLIT_MODE=row
exec python -m torch.distributed.run --standalone --nnodes=1 --nproc-per-node "$N" \
  --local-addr 127.0.0.1 -m llama_fastapi_k8s_gpu_amd.serve
