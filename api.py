"""ASGI entry point kept at the reference's import path so the process server
command is unchanged: ``gunicorn -w 1 -k uvicorn.workers.UvicornWorker api:app``
(reference docker/Dockerfile.app:12)."""
from llama_fastapi_k8s_gpu_amd.server.app import create_app

app = create_app()
