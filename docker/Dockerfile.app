# Service image (reference docker/Dockerfile.app:1-12): the API on top of the
# gfx950 base. One GPU per process: a single-GPU pod runs gunicorn exactly like
# the reference; a pod with N GPUs and SPLIT_MODE=row runs N ranks under torchrun
# (docker/entrypoint.sh picks the launcher from GPUS_PER_POD).
ARG BASE_IMAGE=myregistry/llama-fastapi-mi355x-base:0.1.0
FROM ${BASE_IMAGE}

WORKDIR /app
COPY api.py /app/api.py
COPY docker/entrypoint.sh /app/entrypoint.sh
RUN chmod +x /app/entrypoint.sh && mkdir -p /app/models

EXPOSE 8000
CMD ["/app/entrypoint.sh"]
