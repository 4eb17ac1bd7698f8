"""Process entry point of the service container.

  * one GPU (or CPU): ``python -m llama_fastapi_k8s_gpu_amd.serve`` runs uvicorn on
    the same app object as ``gunicorn -w 1 -k uvicorn.workers.UvicornWorker api:app``
    (reference docker/Dockerfile.app:12);
  * N GPUs, one model (``split_mode=row``):
    ``torchrun --nproc-per-node N -m llama_fastapi_k8s_gpu_amd.serve`` - rank 0
    serves HTTP, ranks 1..N-1 follow (``parallel/tp_serve.py``).

HOST / PORT env (default 0.0.0.0:8000, reference Dockerfile.base EXPOSE 8000).
"""
from __future__ import annotations

import logging
import os


def main() -> int:
    from .config import Settings
    settings = Settings.from_env()
    host = os.environ.get("HOST", "0.0.0.0")
    port = int(os.environ.get("PORT", "8000"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    import uvicorn
    from .server.app import create_app
    if world == 1:
        uvicorn.run(create_app(settings), host=host, port=port, workers=1)
        return 0
    from .engine.factory import build_engine
    from .parallel.tp_serve import TPLeader, follower_loop, init_tp
    rank, world, ctrl = init_tp(settings)
    llm = build_engine(settings)
    native = getattr(llm, "backend_name", "") == "hip"   # the engine mirrors its own commands
    if rank == 0:
        front = llm if native else TPLeader(llm, ctrl)
        try:
            uvicorn.run(create_app(settings, engine=front), host=host, port=port, workers=1)
        finally:
            front.close()
    else:
        logging.getLogger(__name__).info("rank %d/%d following rank 0", rank, world)
        if native:
            llm.follow()
            llm.close()
        else:
            follower_loop(llm, ctrl)
    import torch.distributed as dist
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
