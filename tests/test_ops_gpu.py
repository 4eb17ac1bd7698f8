"""The public torch-facing op wrappers (llama_fastapi_k8s_gpu_amd.ops) vs plain
PyTorch fp32 references of the same ops."""
import numpy as np
import pytest

from gpu_helpers import make_matrix, q8_emulate, rel_err, rmsnorm
from llama_fastapi_k8s_gpu_amd.gguf.constants import GGMLType

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0, GGMLType.Q5_K])
def test_ops_gemv_gemm(torch, t):
    from llama_fastapi_k8s_gpu_amd import ops
    rng = np.random.default_rng(int(t))
    R, K = 384, 1024
    raw, w = make_matrix(t, R, K, rng)
    W = ops.QuantMatrix.from_ggml(raw, t, R, K)
    x = rng.standard_normal(K).astype(np.float32)
    nw = (1 + 0.1 * rng.standard_normal(K)).astype(np.float32)
    xt, nt = torch.from_numpy(x).cuda(), torch.from_numpy(nw).cuda()
    y = ops.gemv(W, xt).cpu().numpy()
    assert rel_err(y, w @ q8_emulate(x)) < 2e-3
    yn = ops.gemv(W, xt, norm=nt).cpu().numpy()
    assert rel_err(yn, w @ q8_emulate(rmsnorm(x, nw))) < 2e-3
    acc = torch.ones(R, device="cuda")
    ops.gemv(W, xt, out=acc, accumulate=True)
    assert rel_err(acc.cpu().numpy(), 1 + w @ q8_emulate(x)) < 2e-3
    X = torch.from_numpy(rng.standard_normal((37, K)).astype(np.float32)).cuda().to(torch.bfloat16)
    Y = ops.gemm(W, X).cpu().numpy()
    ref = X.float().cpu().numpy() @ w.T
    assert rel_err(Y, ref) < 1e-2


def test_ops_swiglu_embed_rmsnorm(torch):
    from llama_fastapi_k8s_gpu_amd import ops
    rng = np.random.default_rng(2)
    F, K = 256, 512
    rg, g = make_matrix(GGMLType.Q4_K, F, K, rng)
    ru, u = make_matrix(GGMLType.Q4_K, F, K, rng)
    W = ops.QuantMatrix.from_ggml(rg, GGMLType.Q4_K, F, K, interleave_gate_up=True, raw_up=ru)
    x = rng.standard_normal(K).astype(np.float32)
    h = ops.gemv_swiglu(W, torch.from_numpy(x).cuda()).cpu().numpy()
    xq = q8_emulate(x)
    a, b = g @ xq, u @ xq
    assert rel_err(h, a / (1 + np.exp(-a)) * b) < 3e-3
    E = ops.QuantMatrix.from_ggml(rg, GGMLType.Q4_K, F, K)
    toks = torch.tensor([0, 5, 255], dtype=torch.int32, device="cuda")
    assert rel_err(ops.embed(E, toks).cpu().numpy(), g[[0, 5, 255]]) < 1e-6
    with pytest.raises(ValueError, match="out of range"):
        ops.embed(E, torch.tensor([256], dtype=torch.int32, device="cuda"))
    X = rng.standard_normal((3, K)).astype(np.float32)
    wn = rng.standard_normal(K).astype(np.float32)
    yb = ops.rmsnorm_bf16(torch.from_numpy(X).cuda(), torch.from_numpy(wn).cuda()).float().cpu().numpy()
    assert rel_err(yb, np.stack([rmsnorm(r, wn) for r in X])) < 1e-2


def test_ops_attention(torch):
    from llama_fastapi_k8s_gpu_amd import ops
    g = torch.Generator(device="cpu").manual_seed(0)
    n_kv, n_ctx, hd, H = 2, 96, 128, 8
    kc = torch.randn(n_kv, n_ctx, hd, generator=g).half().cuda()
    vc = torch.randn(n_kv, n_ctx, hd, generator=g).half().cuda()
    q = torch.randn(H * hd, generator=g).cuda()
    pos = 70
    out = ops.attention_decode(q, kc, vc, pos).cpu()
    K, V = kc.float().cpu(), vc.float().cpu()
    ref = []
    for h in range(H):
        kv = h // (H // n_kv)
        s = (K[kv, :pos + 1] @ q.cpu()[h * hd:(h + 1) * hd]) / hd ** 0.5
        ref.append(torch.softmax(s, 0) @ V[kv, :pos + 1])
    assert rel_err(out.numpy(), torch.cat(ref).numpy()) < 2e-3
    T, pos0 = 5, 20
    Q = torch.randn(T, H * hd, generator=g).cuda()
    outp = ops.attention_prefill(Q, kc, vc, pos0).cpu()
    for t in range(T):
        for h in (0, H - 1):
            kv = h // (H // n_kv)
            L = pos0 + t + 1
            s = (K[kv, :L] @ Q.cpu()[t, h * hd:(h + 1) * hd]) / hd ** 0.5
            r = torch.softmax(s, 0) @ V[kv, :L]
            assert rel_err(outp[t, h * hd:(h + 1) * hd].numpy(), r.numpy()) < 2e-3
    with pytest.raises(ValueError):
        ops.attention_decode(q, kc, vc, n_ctx)          # pos out of range: refused on the host
