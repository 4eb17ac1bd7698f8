"""N1: the ``llama_cpp.Llama``-compatible facade and what it is built from."""
from .cache import LlamaCache, LlamaDeviceCache, LlamaRAMCache, LlamaState  # noqa: F401
