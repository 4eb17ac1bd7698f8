"""Host-side validation of the op wrappers (runs without a GPU: the checks fire
before any launch)."""
import pytest


def test_ops_reject_host_tensors():
    torch = pytest.importorskip("torch")
    from llama_fastapi_k8s_gpu_amd import ops
    W = ops.QuantMatrix(data=None, qtype=12, rows=256, K=256)
    with pytest.raises(ValueError, match="CUDA"):
        ops.gemv(W, torch.zeros(256))
    with pytest.raises(ValueError, match=r"x must be \[T, 256\]"):
        ops.gemm(W, torch.zeros(4, 128, dtype=torch.bfloat16))
