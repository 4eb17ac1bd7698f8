"""MI355X-native GGUF chat service (capabilities of dzatulin/llama-fastapi-k8s-gpu).

Layers:
  server/   N4/N3/N2  FastAPI /response, admission queue, prompt policy
  engine/   N1        Llama-compatible facade, chat templates, tokenizer, sampling
  gguf/               GGUF reader/writer, block quant formats, synthetic models
  models/             model hyper-parameters, torch fp32 reference forward
  runtime/  N0a       native runtime bindings (C++ GPU engine, C++ CPU backend)
  ops/      N0b       HIP kernel wrappers (gfx950)
  parallel/ N0c       tensor-parallel sharding + RCCL bootstrap
  utils/              logging, timers
"""
__version__ = "0.1.0"
