"""T3 - every gfx950 kernel against a plain PyTorch/NumPy fp32 reference of the
same op (shape sweeps include non-multiple-of-tile edges)."""
import numpy as np
import pytest

from llama_fastapi_k8s_gpu_amd.gguf.constants import GGMLType
from gpu_helpers import dev_bytes, hip, make_matrix, q8_emulate, rel_err, rmsnorm, stream, to_planar

pytestmark = pytest.mark.gpu

QTYPES = [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0, GGMLType.F16, GGMLType.F32]


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("t", QTYPES)
@pytest.mark.parametrize("R,K", [(64, 256), (130, 4096), (33, 1024), (96, 14336)])
def test_gemv_types(torch, t, R, K):
    rng = np.random.default_rng(R * K + int(t))
    raw, W = make_matrix(t, R, K, rng)
    x = rng.standard_normal(K).astype(np.float32)
    dw = dev_bytes(to_planar(t, raw, R, K))
    dx = torch.from_numpy(x).cuda()
    out = torch.zeros(R, device="cuda")
    hip().gemv(dw.data_ptr(), int(t), R, K, dx.data_ptr(), 0, 1e-5, out.data_ptr(), R, 0, stream())
    torch.cuda.synchronize()
    ref_q8 = W.astype(np.float64) @ q8_emulate(x).astype(np.float64)
    assert rel_err(out.cpu().numpy(), ref_q8) < 2e-4
    ref = W.astype(np.float64) @ x.astype(np.float64)
    assert rel_err(out.cpu().numpy(), ref) < 2e-2


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("K", [4096, 8192, 28672])   # 8B, 70B d_model, 70B FFN (1024-thread launch paths)
def test_gemv_norm_add_and_resid(torch, t, K):
    rng = np.random.default_rng(7)
    R = 256
    raw, W = make_matrix(t, R, K, rng)
    x = rng.standard_normal(K).astype(np.float32) * 3
    nw = (1 + 0.1 * rng.standard_normal(K)).astype(np.float32)
    dw = dev_bytes(to_planar(t, raw, R, K))
    dx, dn = torch.from_numpy(x).cuda(), torch.from_numpy(nw).cuda()
    y0 = rng.standard_normal(R).astype(np.float32)
    out = torch.from_numpy(y0.copy()).cuda()
    hip().gemv(dw.data_ptr(), int(t), R, K, dx.data_ptr(), dn.data_ptr(), 1e-5, out.data_ptr(), R, 1, stream())
    torch.cuda.synchronize()
    ref = y0 + W @ q8_emulate(rmsnorm(x, nw))
    assert rel_err(out.cpu().numpy() - y0, ref - y0) < 1e-3
    # EPI_STORE with a residual vector
    res = torch.from_numpy(y0.copy()).cuda()
    out2 = torch.zeros(R, device="cuda")
    hip().gemv(dw.data_ptr(), int(t), R, K, dx.data_ptr(), dn.data_ptr(), 1e-5, out2.data_ptr(), R, 0, stream(),
               resid=res.data_ptr())
    torch.cuda.synchronize()
    assert rel_err(out2.cpu().numpy() - y0, ref - y0) < 1e-3


@pytest.mark.parametrize("F,K", [(96, 512), (256, 4096), (128, 8192)])
def test_gemv_swiglu_interleaved(torch, F, K):
    rng = np.random.default_rng(8)
    t = GGMLType.Q4_K
    rg, Wg = make_matrix(t, F, K, rng)
    ru, Wu = make_matrix(t, F, K, rng)
    pg = to_planar(t, rg, F, K, R_dst=2 * F, G=32, off=0)
    pu = to_planar(t, ru, F, K, R_dst=2 * F, G=32, off=32)
    planar = pg | pu  # disjoint rows; the rest is zero in each
    dw = dev_bytes(planar)
    x = rng.standard_normal(K).astype(np.float32)
    dx = torch.from_numpy(x).cuda()
    out = torch.zeros(F, device="cuda")
    hip().gemv(dw.data_ptr(), int(t), 2 * F, K, dx.data_ptr(), 0, 1e-5, out.data_ptr(), F, 2, stream())
    torch.cuda.synchronize()
    xq = q8_emulate(x)
    g, u = Wg @ xq, Wu @ xq
    ref = g / (1 + np.exp(-g)) * u
    assert rel_err(out.cpu().numpy(), ref) < 1e-3


def test_gemv_moe_slots_and_down(torch):
    rng = np.random.default_rng(9)
    E, F, K, d = 4, 256, 256, 128
    t = GGMLType.Q4_K
    mats = [(make_matrix(t, F, K, rng), make_matrix(t, F, K, rng)) for _ in range(E)]
    planar = []
    for (rg, Wg), (ru, Wu) in mats:
        planar.append(to_planar(t, rg, F, K, R_dst=2 * F, G=32, off=0) | to_planar(t, ru, F, K, R_dst=2 * F, G=32, off=32))
    stride = planar[0].size
    dw = dev_bytes(np.concatenate(planar))
    x = rng.standard_normal(K).astype(np.float32)
    dx = torch.from_numpy(x).cuda()
    ids = torch.tensor([3, 1], dtype=torch.int32, device="cuda")
    out = torch.zeros(2, F, device="cuda")
    hip().gemv(dw.data_ptr(), int(t), 2 * F, K, dx.data_ptr(), 0, 1e-5, out.data_ptr(), F, 2, stream(),
               n_slots=2, ids=ids.data_ptr(), expert_stride=stride, slot_stride=F)
    torch.cuda.synchronize()
    xq = q8_emulate(x)
    for s, e in enumerate([3, 1]):
        g, u = mats[e][0][1] @ xq, mats[e][1][1] @ xq
        assert rel_err(out[s].cpu().numpy(), g / (1 + np.exp(-g)) * u) < 1e-3
    # down projection, weighted over the two slots
    downs = [make_matrix(t, d, F, rng) for _ in range(E)]
    dd = dev_bytes(np.concatenate([to_planar(t, r, d, F) for r, _ in downs]))
    h = rng.standard_normal((2, F)).astype(np.float32)
    dh = torch.from_numpy(h).cuda()
    wts = torch.tensor([0.7, 0.3], device="cuda")
    y = torch.ones(d, device="cuda")
    hip().moe_down(dd.data_ptr(), int(t), d, F, to_planar(t, downs[0][0], d, F).size, dh.data_ptr(), ids.data_ptr(),
                   wts.data_ptr(), 2, y.data_ptr(), stream())
    torch.cuda.synchronize()
    ref = 1 + 0.7 * downs[3][1] @ q8_emulate(h[0]) + 0.3 * downs[1][1] @ q8_emulate(h[1])
    assert rel_err(y.cpu().numpy() - 1, ref - 1) < 1e-3


def test_moe_route(torch):
    logits = torch.tensor([0.1, 2.0, -1.0, 1.5, 0.3, 0.0, -2.0, 1.9], device="cuda")
    ids = torch.zeros(2, dtype=torch.int32, device="cuda")
    w = torch.zeros(2, device="cuda")
    hip().moe_route(logits.data_ptr(), 8, 2, ids.data_ptr(), w.data_ptr(), stream())
    torch.cuda.synchronize()
    assert ids.tolist() == [1, 7]
    p = torch.softmax(logits.cpu(), 0)
    np.testing.assert_allclose(w.cpu().numpy(), (p[[1, 7]] / p[[1, 7]].sum()).numpy(), rtol=1e-5)


@pytest.mark.parametrize("E,k,d,B", [(8, 2, 4096, 6), (8, 2, 4096, 1), (16, 4, 2048, 3), (8, 2, 8192, 8)])
def test_moe_router_rows_vs_fp64(torch, E, k, d, B):
    """The batched decode router (one block per row: f32 RMSNorm(x) * w . W^T, softmax, top-k,
    renormalised, as a dense [B][E] weight row, zeros for the unrouted experts) against an fp64
    reference; the columns past E are untouched."""
    rng = np.random.default_rng(E * 100 + d + B)
    ldx = d + 8
    x = torch.from_numpy(rng.standard_normal((B, ldx)).astype(np.float32)).cuda()
    nw = torch.from_numpy((1 + 0.1 * rng.standard_normal(d)).astype(np.float32)).cuda()
    W = torch.from_numpy((0.05 * rng.standard_normal((E, d))).astype(np.float32)).cuda()
    ld = E + 3
    one = torch.full((B, ld), 7.0, device="cuda")
    hip().moe_router_rows(x.data_ptr(), ldx, B, nw.data_ptr(), 1e-5, W.data_ptr(), d, E, k, one.data_ptr(), ld,
                          stream())
    torch.cuda.synchronize()
    xs = x.cpu().numpy()[:, :d].astype(np.float64)
    n = xs / np.sqrt((xs ** 2).mean(1, keepdims=True) + 1e-5) * nw.cpu().numpy()
    lg = n @ W.cpu().numpy().astype(np.float64).T
    p = np.exp(lg - lg.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    got = one.cpu().numpy()
    for b in range(B):
        top = np.argsort(-p[b], kind="stable")[:k]
        ref = np.zeros(E)
        ref[top] = p[b][top] / p[b][top].sum()
        np.testing.assert_allclose(got[b, :E], ref, rtol=1e-4, atol=1e-6)
        assert np.all(got[b, E:] == 7.0)


@pytest.mark.parametrize("tq,tk,tv", [(GGMLType.Q4_K, GGMLType.Q4_K, GGMLType.Q6_K),   # two runs, one launch
                                      (GGMLType.Q4_K, GGMLType.Q8_0, GGMLType.Q8_0),
                                      (GGMLType.Q4_K, GGMLType.Q4_K, GGMLType.Q4_K),   # one run
                                      (GGMLType.Q6_K, GGMLType.Q4_K, GGMLType.Q6_K)])  # three runs: per-segment
@pytest.mark.parametrize("K", [512, 8192])   # 8192: the one-CU launch path (K > 4096, 70B)
def test_gemv_qkv_rope_kvstore(torch, tq, tk, tv, K):
    rng = np.random.default_rng(10)
    hd, nh, nkv, n_ctx, pos = 64, 8, 2, 32, 5
    (rq, Wq), (rk, Wk), (rv, Wv) = make_matrix(tq, nh * hd, K, rng), make_matrix(tk, nkv * hd, K, rng), \
        make_matrix(tv, nkv * hd, K, rng)
    dq, dk, dv = (dev_bytes(to_planar(t, r, R, K)) for t, r, R in ((tq, rq, nh * hd), (tk, rk, nkv * hd), (tv, rv, nkv * hd)))
    x = rng.standard_normal(K).astype(np.float32)
    nw = np.ones(K, np.float32)
    dx, dn = torch.from_numpy(x).cuda(), torch.from_numpy(nw).cuda()
    qo = torch.zeros(nh * hd, device="cuda")
    kc = torch.zeros(nkv, n_ctx, hd, dtype=torch.float16, device="cuda")
    vc = torch.zeros_like(kc)
    dpos = torch.tensor([pos], dtype=torch.int32, device="cuda")
    inv = 10000.0 ** (-2 * np.arange(hd // 2) / hd)
    ang = np.arange(n_ctx)[:, None] * inv[None]
    rope = torch.from_numpy(np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32)).cuda()
    hip().gemv_qkv(dq.data_ptr(), int(tq), dk.data_ptr(), int(tk), dv.data_ptr(), int(tv), nh * hd, nkv * hd, K,
                   dx.data_ptr(), dn.data_ptr(), 1e-5, qo.data_ptr(), kc.data_ptr(), vc.data_ptr(), n_ctx, hd,
                   dpos.data_ptr(), rope.data_ptr(), stream())
    torch.cuda.synchronize()
    xq = q8_emulate(rmsnorm(x, nw))

    def rot(v):
        v = v.reshape(-1, hd)
        c, s = np.cos(ang[pos]), np.sin(ang[pos])
        o = v.copy()
        o[:, 0::2] = v[:, 0::2] * c - v[:, 1::2] * s
        o[:, 1::2] = v[:, 0::2] * s + v[:, 1::2] * c
        return o
    assert rel_err(qo.cpu().numpy().reshape(nh, hd), rot(Wq @ xq)) < 1e-3
    assert rel_err(kc[:, pos].float().cpu().numpy(), rot(Wk @ xq)) < 2e-3
    assert rel_err(vc[:, pos].float().cpu().numpy(), (Wv @ xq).reshape(nkv, hd)) < 2e-3
    assert float(kc[:, pos + 1].abs().sum()) == 0.0


def _attn_ref(q, K, V, L, scale):
    # q [H, D], K/V [Hkv, L, D]
    H, D = q.shape
    G = H // K.shape[0]
    out = np.zeros((H, D))
    for h in range(H):
        k = K[h // G, :L].astype(np.float64)
        s = k @ q[h].astype(np.float64) * scale
        p = np.exp(s - s.max())
        p /= p.sum()
        out[h] = p @ V[h // G, :L].astype(np.float64)
    return out


@pytest.mark.parametrize("hd,H,Hkv", [(128, 32, 8), (64, 32, 4)])
@pytest.mark.parametrize("L", [1, 31, 64, 65, 1000])
def test_attn_decode(torch, hd, H, Hkv, L):
    rng = np.random.default_rng(L + hd)
    n_ctx = 1024
    q = rng.standard_normal((H, hd)).astype(np.float32)
    K = rng.standard_normal((Hkv, n_ctx, hd)).astype(np.float16)
    V = rng.standard_normal((Hkv, n_ctx, hd)).astype(np.float16)
    dq = torch.from_numpy(q).cuda()
    dK, dV = torch.from_numpy(K).cuda(), torch.from_numpy(V).cuda()
    pos = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
    ws = torch.zeros(hip().attn_decode_workspace_floats(n_ctx, H, hd), device="cuda")
    out = torch.zeros(H, hd, device="cuda")
    stride, xcds, n_ints = hip().chain_layout()
    cnt = torch.zeros(n_ints, dtype=torch.int32, device="cuda")
    scale = 1 / np.sqrt(hd)
    for _ in range(3):  # repeated launches: counters must return to zero
        out.zero_()
        hip().attn_decode(dq.data_ptr(), dK.data_ptr(), dV.data_ptr(), pos.data_ptr(), n_ctx, H, Hkv, hd, scale,
                          ws.data_ptr(), out.data_ptr(), stream(), cnt.data_ptr())
        torch.cuda.synchronize()
        # q*scale is rounded to f16 for the v_dot2 score path (upstream's KQ is f16 too)
        assert rel_err(out.cpu().numpy(), _attn_ref(q, K, V, L, scale)) < 3e-3
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("T,pos0", [(1, 0), (17, 0), (40, 23), (130, 0), (200, 301)])
@pytest.mark.parametrize("H,Hkv", [(8, 2), (8, 8), (16, 2), (8, 4), (6, 2)])
def test_attn_prefill(torch, hd, T, pos0, H, Hkv):
    """MFMA flash prefill (GQA group 1/2/4/8) and the scalar fallback (group 3) vs fp64."""
    rng = np.random.default_rng(T + pos0 + 7 * H + Hkv)
    n_ctx = 512
    q = rng.standard_normal((T, H, hd)).astype(np.float32)
    K = rng.standard_normal((Hkv, n_ctx, hd)).astype(np.float16)
    V = rng.standard_normal((Hkv, n_ctx, hd)).astype(np.float16)
    out = torch.zeros(T, H, hd, device="cuda")
    scale = 1 / np.sqrt(hd)
    dq, dK, dV = (torch.from_numpy(a).cuda() for a in (q, K, V))  # keep the device copies alive
    hip().attn_prefill(dq.data_ptr(), dK.data_ptr(), dV.data_ptr(), T, pos0, n_ctx, H, Hkv, hd, scale,
                       out.data_ptr(), stream())
    torch.cuda.synchronize()
    ref = np.stack([_attn_ref(q[t], K, V, pos0 + t + 1, scale) for t in range(T)])
    # the MFMA path rounds q*scale and the softmax weights to f16 (upstream's KQ/KQV are f16 too)
    assert rel_err(out.cpu().numpy(), ref) < (1e-4 if H // Hkv == 3 else 3e-3)
    if H // Hkv != 3:  # bf16 output (what the engine feeds the Wo GEMM)
        ob = torch.zeros(T, H, hd, device="cuda", dtype=torch.bfloat16)
        hip().attn_prefill(dq.data_ptr(), dK.data_ptr(), dV.data_ptr(), T, pos0, n_ctx, H, Hkv, hd, scale,
                           ob.data_ptr(), stream(), True)
        torch.cuda.synchronize()
        assert rel_err(ob.float().cpu().numpy(), ref) < 8e-3
        # f16 in bmm's 4-group k order (the tile16 prefill GEMM's input)
        oh = torch.zeros(T, H * hd, device="cuda", dtype=torch.float16)
        hip().attn_prefill(dq.data_ptr(), dK.data_ptr(), dV.data_ptr(), T, pos0, n_ctx, H, Hkv, hd, scale,
                           oh.data_ptr(), stream(), out_h=True)
        torch.cuda.synchronize()
        got = _swizzle4(oh.float().cpu().numpy()).reshape(T, H, hd)
        assert rel_err(got, ref) < 3e-3


@pytest.mark.parametrize("t", QTYPES)
@pytest.mark.parametrize("T,N,K", [(1, 128, 256), (33, 256, 512), (130, 384, 1024), (300, 256, 2048)])
def test_gemm_mfma(torch, t, T, N, K):
    rng = np.random.default_rng(T * N + int(t))
    raw, W = make_matrix(t, N, K, rng)
    dw = dev_bytes(to_planar(t, raw, N, K))
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    out = torch.zeros(T, N, device="cuda")
    hip().gemm(dw.data_ptr(), int(t), N, K, x.data_ptr(), T, out.data_ptr(), 0, N, 0, stream())
    torch.cuda.synchronize()
    Wb = torch.from_numpy(W).to(torch.bfloat16).float()  # the kernel stages weights as bf16
    ref = x.float().cpu() @ Wb.T
    assert rel_err(out.cpu().numpy(), ref.numpy()) < 5e-3
    # residual-add epilogue
    base = torch.randn(T, N, device="cuda")
    acc = base.clone()
    hip().gemm(dw.data_ptr(), int(t), N, K, x.data_ptr(), T, acc.data_ptr(), 0, N, 1, stream())
    torch.cuda.synchronize()
    assert rel_err((acc - base).cpu().numpy(), ref.numpy()) < 5e-3


@pytest.mark.parametrize("T", [40, 70, 200])   # 64-token tiles, and 128-token tiles (one / two, partial)
def test_gemm_swiglu(torch, T):
    rng = np.random.default_rng(11)
    F, K = 128, 512
    t = GGMLType.Q4_K
    rg, Wg = make_matrix(t, F, K, rng)
    ru, Wu = make_matrix(t, F, K, rng)
    planar = to_planar(t, rg, F, K, R_dst=2 * F, G=32, off=0) | to_planar(t, ru, F, K, R_dst=2 * F, G=32, off=32)
    dw = dev_bytes(planar)
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    h = torch.zeros(T, F, dtype=torch.bfloat16, device="cuda")
    hip().gemm(dw.data_ptr(), int(t), 2 * F, K, x.data_ptr(), T, 0, h.data_ptr(), 0, 2, stream())
    torch.cuda.synchronize()
    xf = x.float().cpu().numpy()
    g = xf @ torch.from_numpy(Wg).to(torch.bfloat16).float().numpy().T
    u = xf @ torch.from_numpy(Wu).to(torch.bfloat16).float().numpy().T
    ref = g / (1 + np.exp(-g)) * u
    assert rel_err(h.float().cpu().numpy(), ref) < 1e-2


@pytest.mark.parametrize("t", QTYPES)
def test_embed(torch, t):
    rng = np.random.default_rng(12)
    V, d = 300, 256
    raw, W = make_matrix(t, V, d, rng)
    dw = dev_bytes(to_planar(t, raw, V, d))
    toks = torch.tensor([0, 5, 299, 17], dtype=torch.int32, device="cuda")
    x = torch.zeros(4, d, device="cuda")
    hip().embed(dw.data_ptr(), int(t), V, d, toks.data_ptr(), 4, x.data_ptr(), stream())
    torch.cuda.synchronize()
    np.testing.assert_allclose(x.cpu().numpy(), W[[0, 5, 299, 17]], rtol=1e-5, atol=1e-6)


def test_rmsnorm_bf16(torch):
    x = torch.randn(5, 4096, device="cuda")
    w = torch.rand(4096, device="cuda") + 0.5
    y = torch.zeros(5, 4096, dtype=torch.bfloat16, device="cuda")
    hip().rmsnorm_bf16(x.data_ptr(), w.data_ptr(), 1e-5, 5, 4096, y.data_ptr(), stream())
    torch.cuda.synchronize()
    ref = x * torch.rsqrt((x * x).mean(-1, keepdim=True) + 1e-5) * w
    assert rel_err(y.float().cpu().numpy(), ref.cpu().numpy()) < 5e-3


def _run_sampler(torch, logits, ring_tokens, params, seed, step=0):
    h = hip()
    V = logits.shape[0]
    dl = torch.from_numpy(logits).cuda()
    pb = np.frombuffer(h.sampler_params_bytes(params.top_k, params.top_p, params.min_p, params.temperature,
                                              params.repeat_penalty, params.frequency_penalty,
                                              params.presence_penalty, params.last_n, seed,
                                              int(params.temperature <= 0), params.tfs_z, params.typical_p,
                                              dict(params.logit_bias)), np.uint8)
    dp = torch.from_numpy(pb.copy()).cuda()
    ring = np.zeros(64, np.int32)
    rl = min(len(ring_tokens), 64)
    ring[:rl] = ring_tokens[-rl:] if rl else []
    state = np.zeros(8, np.int32)
    state[2] = step
    state[3] = rl
    state[4] = rl & 63
    dr, ds = torch.from_numpy(ring).cuda(), torch.from_numpy(state).cuda()
    cand = torch.zeros(h.sampler_cand_words(V), dtype=torch.int32, device="cuda")
    h.sample(dl.data_ptr(), V, dp.data_ptr(), dr.data_ptr(), ds.data_ptr(), cand.data_ptr(), 0, 0, 1, stream())
    torch.cuda.synchronize()
    return int(ds[0].item()), ds.cpu().numpy()


def test_sampler_greedy_with_penalties(torch):
    from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams, apply_penalties
    rng = np.random.default_rng(13)
    logits = rng.standard_normal(128256).astype(np.float32) * 4
    top = int(np.argmax(logits))
    p = SamplingParams(temperature=0.0, top_k=1, repeat_penalty=1.5, frequency_penalty=2.0, presence_penalty=1.0)
    tok, st = _run_sampler(torch, logits, [top, top, 7], p, 0)
    assert tok == int(np.argmax(apply_penalties(logits, [top, top, 7], p)))
    assert st[1] == 1 and st[2] == 1  # pos and step advanced


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sampler_vocab_parallel_equals_single(torch, world):
    """Tensor-parallel sampling: stage 1 on each vocabulary shard (global ids offset, equal
    slice counts), the shards' candidate blocks concatenated as the all-gather leaves them,
    stage 2 on the gathered blocks == the one-shard sampler (same token, same state)."""
    from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams
    h = hip()
    rng = np.random.default_rng(20 + world)
    for it in range(6):
        V = [128256, 32000, 1000][it % 3]
        logits = (rng.standard_normal(V) * 3).astype(np.float32)
        hist = [int(t) for t in rng.integers(0, V, 70)]
        p = SamplingParams(temperature=1.2, top_k=40, top_p=0.9, min_p=0.05, repeat_penalty=1.1,
                           frequency_penalty=0.7, presence_penalty=0.8, seed=7 + it,
                           logit_bias={int(hist[3]): 2.5, 5: -1.0})
        want, want_st = _run_sampler(torch, logits, hist, p, p.seed, step=it)
        pb = np.frombuffer(h.sampler_params_bytes(p.top_k, p.top_p, p.min_p, p.temperature, p.repeat_penalty,
                                                  p.frequency_penalty, p.presence_penalty, p.last_n, p.seed, 0,
                                                  p.tfs_z, p.typical_p, dict(p.logit_bias)), np.uint8)
        dp = torch.from_numpy(pb.copy()).cuda()
        V_l = (V + world - 1) // world
        W = h.sampler_cand_words(V_l)
        gathered = torch.zeros(world * W, dtype=torch.int32, device="cuda")
        ring = np.zeros(64, np.int32)
        ring[:64] = hist[-64:]
        states = []
        for r in range(world):
            shard = np.zeros(V_l, np.float32)
            n = max(0, min(V_l, V - r * V_l))
            shard[:n] = logits[r * V_l:r * V_l + n]
            dl = torch.from_numpy(shard).cuda()
            st = np.zeros(8, np.int32)
            st[2], st[3], st[4] = it, 64, 0
            ds, dr = torch.from_numpy(st).cuda(), torch.from_numpy(ring.copy()).cuda()
            h.sample(dl.data_ptr(), n, dp.data_ptr(), dr.data_ptr(), ds.data_ptr(),
                     gathered[r * W:(r + 1) * W].data_ptr(), 0, 0, 1, stream(), vocab_off=r * V_l, V_glob=V,
                     V_span=V_l, stage=1)
            states.append((ds, dr, dl))
        torch.cuda.synchronize()
        for ds, dr, dl in states:   # every rank runs the identical stage 2
            h.sample(dl.data_ptr(), V_l, dp.data_ptr(), dr.data_ptr(), ds.data_ptr(), gathered.data_ptr(), 0, 0, 1,
                     stream(), vocab_off=0, V_glob=V, V_span=V_l, cand_all=gathered.data_ptr(), world=world, stage=2)
        torch.cuda.synchronize()
        for ds, _, _ in states:
            assert int(ds[0].item()) == want, (world, it, int(ds[0].item()), want)
            assert (ds.cpu().numpy()[:6] == want_st[:6]).all()


def test_sampler_matches_host_chain(torch):
    from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams, filtered_candidates, sample_token
    rng = np.random.default_rng(14)
    agree = outside = 0
    n = 40
    for i in range(n):
        V = [32000, 128256, 1000][i % 3]
        logits = (rng.standard_normal(V) * 3).astype(np.float32)
        hist = list(rng.integers(0, V, 80))
        p = SamplingParams(temperature=1.2, top_k=40, top_p=0.9, min_p=0.05, repeat_penalty=1.1,
                           frequency_penalty=0.7, presence_penalty=0.8, seed=1000 + i)
        tok, _ = _run_sampler(torch, logits, hist, p, p.seed, step=i)
        ids, _ = filtered_candidates(logits, hist[-64:], p)
        # f32 (GPU) vs f64 (host) can move a top-p / min-p boundary by one candidate
        outside += tok not in set(ids.tolist())
        agree += tok == sample_token(logits, hist[-64:], p, i)
    assert outside <= 2
    assert agree >= n - 3


def _chi2_logits(V=32000):
    # 12 live candidates with spread logits, the rest far below (top-p / top-k cut inside the live set)
    rng = np.random.default_rng(21)
    logits = np.full(V, -30.0, np.float32) + rng.standard_normal(V).astype(np.float32)
    live = rng.choice(V, 12, replace=False)
    logits[live] = np.linspace(4.0, 0.5, 12).astype(np.float32)
    return logits, live


def test_sampler_distribution_chi2(torch):
    """T5: the GPU draw follows the host chain's distribution (penalties -> top-k -> top-p
    -> min-p -> temperature) - chi-square over 3000 draws with independent Philox streams."""
    from scipy.stats import chisquare
    from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams, _softmax, filtered_candidates
    logits, live = _chi2_logits()
    hist = [int(live[0]), int(live[0]), int(live[3]), 5, 6]
    p = SamplingParams(temperature=1.2, top_k=40, top_p=0.95, min_p=0.0, repeat_penalty=1.0,
                       frequency_penalty=0.7, presence_penalty=0.8)
    ids, vals = filtered_candidates(logits, hist, p)
    probs = _softmax(vals.astype(np.float64))
    index = {int(t): j for j, t in enumerate(ids)}
    counts = np.zeros(len(ids))
    n = 3000
    for s in range(n):
        tok, _ = _run_sampler(torch, logits, hist, p, 7919 * s + 3, step=s)
        assert tok in index, tok  # never outside the filtered set
        counts[index[tok]] += 1
    exp = probs * n
    keep = exp >= 5  # standard chi-square validity; pool the thin tail
    f_obs = np.append(counts[keep], counts[~keep].sum())
    f_exp = np.append(exp[keep], exp[~keep].sum())
    if f_exp[-1] == 0:
        f_obs, f_exp = f_obs[:-1], f_exp[:-1]
    assert chisquare(f_obs, f_exp * f_obs.sum() / f_exp.sum()).pvalue > 1e-3, (counts, exp)


@pytest.mark.parametrize("mode", ["tfs", "typical", "bias", "all"])
def test_sampler_tail_free_typical_bias_match_host_chain(torch, mode):
    """Tail-free, locally-typical and logit bias on the device (stage 2 on the sorted <= 64
    candidates; bias in stage 1 before the penalties) vs the host chain."""
    from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams, filtered_candidates, sample_token
    rng = np.random.default_rng({"tfs": 31, "typical": 32, "bias": 33, "all": 34}[mode])
    agree = outside = 0
    n = 30
    for i in range(n):
        V = [32000, 128256, 1000][i % 3]
        logits = (rng.standard_normal(V) * 3).astype(np.float32)
        hist = list(rng.integers(0, V, 80))
        kw = {}
        if mode in ("tfs", "all"):
            kw["tfs_z"] = 0.9
        if mode in ("typical", "all"):
            kw["typical_p"] = 0.8
        if mode in ("bias", "all"):
            top = np.argsort(-logits)[:3]
            kw["logit_bias"] = {int(top[0]): -2.5, int(rng.integers(0, V)): 6.0, int(hist[-1]): 1.5}
        p = SamplingParams(temperature=1.1, top_k=40, top_p=0.95, min_p=0.02, repeat_penalty=1.1,
                           frequency_penalty=0.5, presence_penalty=0.3, seed=500 + i, **kw)
        tok, _ = _run_sampler(torch, logits, hist, p, p.seed, step=i)
        ids, _ = filtered_candidates(logits, hist[-64:], p)
        outside += tok not in set(ids.tolist())
        agree += tok == sample_token(logits, hist[-64:], p, i)
    assert outside <= 2, outside
    assert agree >= n - 3, agree


def test_sampler_bias_greedy_forces_and_bans(torch):
    from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams
    rng = np.random.default_rng(40)
    logits = rng.standard_normal(128256).astype(np.float32)
    top = int(np.argmax(logits))
    p = SamplingParams(temperature=0.0, top_k=1, repeat_penalty=1.0, logit_bias={128255: 50.0})
    assert _run_sampler(torch, logits, [], p, 0)[0] == 128255
    p = SamplingParams(temperature=0.0, top_k=1, repeat_penalty=1.0, logit_bias={top: float("-inf")})
    tok = _run_sampler(torch, logits, [], p, 0)[0]
    assert tok != top and tok == int(np.argsort(-logits)[1])



BM_TYPES = [GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.Q8_0]


def _swizzle4(x):
    """bprep's k order inside each 4-group: (0, 2, 1, 3)."""
    return x.reshape(*x.shape[:-1], -1, 4)[..., [0, 2, 1, 3]].reshape(x.shape)


@pytest.mark.parametrize("t", BM_TYPES)
@pytest.mark.parametrize("B", [1, 3, 8, 16])
@pytest.mark.parametrize("R,K", [(130, 4096), (48, 14336), (16, 256)])
def test_bmm_rows_vs_fp32(torch, t, B, R, K):
    """MFMA batched projection: out[b] += W x[b] for every row b, against the fp32 product
    with the f16 activations; partials accumulate onto the existing output."""
    rng = np.random.default_rng(B * 1000 + R + int(t))
    raw, W = make_matrix(t, R, K, rng)
    dw = dev_bytes(to_planar(t, raw, R, K))
    X = rng.standard_normal((B, K)).astype(np.float32)
    Xh = X.astype(np.float16)
    y0 = rng.standard_normal((B, R)).astype(np.float32)
    ldo = R + 6
    out = torch.zeros(B, ldo, device="cuda")
    out[:, :R] = torch.from_numpy(y0).cuda()
    dxh = torch.from_numpy(_swizzle4(Xh)).cuda()   # keep device buffers referenced until the kernel ran
    tw = torch.empty(hip().t16_bytes(int(t), R, K), dtype=torch.uint8, device="cuda")
    hip().t16_repack(dw.data_ptr(), int(t), R, K, tw.data_ptr(), stream())
    hip().bmm(tw.data_ptr(), int(t), R, K, dxh.data_ptr(), K, out.data_ptr(), ldo, B, stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ref = Xh.astype(np.float64) @ W.astype(np.float64).T
    for b in range(B):
        assert rel_err(got[b, :R] - y0[b], ref[b]) < 2e-3, (b, rel_err(got[b, :R] - y0[b], ref[b]))
        assert np.all(got[b, R:] == 0)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("B", [1, 5, 8])
@pytest.mark.parametrize("F,K", [(256, 4096), (96, 2048), (7168, 4096)])
def test_bmm_swiglu_epilogue_vs_fp32(torch, t, B, F, K):
    """Gate/up projection with the SwiGLU epilogue: W rows in 32-row gate / up groups, regrouped
    by the SwiGLU tile16 copy into 8 gate + 8 up rows per tile; the kernel writes silu(gate) * up
    as f16 in bprep's (0, 2, 1, 3) 4-group order, against the fp32 product of the same f16
    activations. F = 7168 (the 8B's TP=2 slice): 896 tiles over the per-CU balanced ranges."""
    rng = np.random.default_rng(B * 100 + F + int(t))
    R = 2 * F
    raw, W = make_matrix(t, R, K, rng)
    dw = dev_bytes(to_planar(t, raw, R, K))
    X = rng.standard_normal((B, K)).astype(np.float32)
    Xh = X.astype(np.float16)
    dxh = torch.from_numpy(_swizzle4(Xh)).cuda()
    ldh_out = F + 8
    hout = torch.full((B, ldh_out), 7.0, dtype=torch.float16, device="cuda")
    tw = torch.empty(hip().t16_bytes(int(t), R, K), dtype=torch.uint8, device="cuda")
    hip().t16_repack(dw.data_ptr(), int(t), R, K, tw.data_ptr(), stream(), swiglu=True)
    hip().bmm(tw.data_ptr(), int(t), R, K, dxh.data_ptr(), K, 0, 0, B, stream(),
              h_out=hout.data_ptr(), ldh_out=ldh_out)
    torch.cuda.synchronize()
    got = hout.cpu().numpy().astype(np.float64)
    pre = Xh.astype(np.float64) @ W.astype(np.float64).T          # [B][2F]
    g = pre.reshape(B, F // 32, 2, 32)[:, :, 0].reshape(B, F)
    u = pre.reshape(B, F // 32, 2, 32)[:, :, 1].reshape(B, F)
    ref = g / (1.0 + np.exp(-g)) * u
    for b in range(B):
        row = _swizzle4(got[b, :F][None])[0]   # the swizzle is its own inverse
        assert rel_err(row, ref[b]) < 3e-3, (b, rel_err(row, ref[b]))
        assert np.all(got[b, F:] == 7.0)


@pytest.mark.parametrize("td", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("B", [1, 6])
@pytest.mark.parametrize("norm", [False, True])
def test_bmm_ffn_chain_matches_two_launches(torch, td, B, norm):
    """The gate/up + down chain in ONE launch (bmm_ffn_chain: down blocks wait per K part on the
    gate/up tiles they read, then stage them with sc1 loads) against the same two projections as
    separate launches, on the 8B FFN shape: the SwiGLU rows bit-identical, the down sums equal up
    to the split-K atomics' order. Run three times over the same counters' fresh zeros."""
    rng = np.random.default_rng(B * 10 + int(td) + norm)
    F, K = 14336, 4096
    raw_g, _ = make_matrix(GGMLType.Q4_K, 2 * F, K, rng)
    raw_d, _ = make_matrix(td, K, F, rng)
    dwg = dev_bytes(to_planar(GGMLType.Q4_K, raw_g, 2 * F, K))
    dwd = dev_bytes(to_planar(td, raw_d, K, F))
    tg = torch.empty(hip().t16_bytes(int(GGMLType.Q4_K), 2 * F, K), dtype=torch.uint8, device="cuda")
    tdw = torch.empty(hip().t16_bytes(int(td), K, F), dtype=torch.uint8, device="cuda")
    hip().t16_repack(dwg.data_ptr(), int(GGMLType.Q4_K), 2 * F, K, tg.data_ptr(), stream(), swiglu=True)
    hip().t16_repack(dwd.data_ptr(), int(td), K, F, tdw.data_ptr(), stream(), swiglu=False)
    X = rng.standard_normal((B, K)).astype(np.float32)
    dxh = torch.from_numpy(_swizzle4(X.astype(np.float16))).cuda()
    dxf = torch.from_numpy(X * 3).cuda()
    nw = torch.from_numpy((0.5 + rng.random(K)).astype(np.float32)).cuda()
    resid = torch.from_numpy(rng.standard_normal((B, K)).astype(np.float32)).cuda()
    xf_ptr, norm_ptr = (dxf.data_ptr(), nw.data_ptr()) if norm else (0, 0)
    # reference: the two launches
    h_ref = torch.zeros(B, F, dtype=torch.float16, device="cuda")
    out_ref = resid.clone()
    hip().bmm(tg.data_ptr(), int(GGMLType.Q4_K), 2 * F, K, dxh.data_ptr(), K, 0, 0, B, stream(),
              h_out=h_ref.data_ptr(), ldh_out=F, xf=xf_ptr, ldxf=K if norm else 0, norm=norm_ptr, eps=1e-5)
    hip().bmm(tdw.data_ptr(), int(td), K, F, h_ref.data_ptr(), F, out_ref.data_ptr(), K, B, stream())
    torch.cuda.synchronize()
    stride, xcds, n_ints = hip().chain_layout()
    cnt = torch.zeros(n_ints, dtype=torch.int32, device="cuda")
    for _ in range(3):
        cnt.zero_()
        h = torch.full((B, F), 3.0, dtype=torch.float16, device="cuda")
        out = resid.clone()
        hip().bmm_ffn_chain(tg.data_ptr(), int(GGMLType.Q4_K), F, K, dxh.data_ptr(), xf_ptr, norm_ptr, 1e-5,
                            tdw.data_ptr(), int(td), h.data_ptr(), out.data_ptr(), B, cnt.data_ptr(), stream())
        torch.cuda.synchronize()
        assert torch.equal(h, h_ref)
        assert rel_err(out.cpu().numpy() - resid.cpu().numpy(), out_ref.cpu().numpy() - resid.cpu().numpy()) < 1e-5
        # every K part counted all of its 224 gate/up tiles
        c = cnt.cpu().numpy()
        per_part = c.reshape(-1, xcds, stride)[:, :, 0].sum(1)
        assert per_part[:8].tolist() == [224] * 8 and not per_part[8:-1].any(), per_part
        # the last part counts the gate/up blocks that staged their x (one per block)
        assert per_part[-1] > 0 and c.sum() == 8 * 224 + per_part[-1], per_part


@pytest.mark.parametrize("td", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("B", [1, 6])
def test_bmm_wo_ffn_chain_matches_three_launches(torch, td, B):
    """Wo -> gate/up -> down in ONE launch (bmm_wo_ffn_chain: the gate/up blocks wait until every Wo
    block has added its split-K partials into the residual rows, stage norm(rows) with sc1 loads; the
    down blocks wait per K part and until every gate/up block has read its rows, then add into them)
    against the three projections as separate launches on the 8B shapes. Three runs over fresh zeros."""
    rng = np.random.default_rng(B * 7 + int(td))
    F, K = 14336, 4096
    raw_o, _ = make_matrix(GGMLType.Q4_K, K, K, rng)
    raw_g, _ = make_matrix(GGMLType.Q4_K, 2 * F, K, rng)
    raw_d, _ = make_matrix(td, K, F, rng)
    mats = []
    for t, R, C, raw, sw in ((GGMLType.Q4_K, K, K, raw_o, False), (GGMLType.Q4_K, 2 * F, K, raw_g, True),
                             (td, K, F, raw_d, False)):
        dw = dev_bytes(to_planar(t, raw, R, C))
        tw = torch.empty(hip().t16_bytes(int(t), R, C), dtype=torch.uint8, device="cuda")
        hip().t16_repack(dw.data_ptr(), int(t), R, C, tw.data_ptr(), stream(), swiglu=sw)
        mats.append(tw)
    to_, tg, tdw = mats
    XA = rng.standard_normal((B, K)).astype(np.float32)
    dxa = torch.from_numpy(_swizzle4(XA.astype(np.float16))).cuda()
    resid0 = torch.from_numpy((rng.standard_normal((B, K)) * 2).astype(np.float32)).cuda()
    nw = torch.from_numpy((0.5 + rng.random(K)).astype(np.float32)).cuda()
    xh = torch.zeros(B, K, dtype=torch.float16, device="cuda")  # (unused: the norm path stages resid)
    # reference: three launches
    r_ref = resid0.clone()
    h_ref = torch.zeros(B, F, dtype=torch.float16, device="cuda")
    hip().bmm(to_.data_ptr(), int(GGMLType.Q4_K), K, K, dxa.data_ptr(), K, r_ref.data_ptr(), K, B, stream())
    hip().bmm(tg.data_ptr(), int(GGMLType.Q4_K), 2 * F, K, xh.data_ptr(), K, 0, 0, B, stream(),
              h_out=h_ref.data_ptr(), ldh_out=F, xf=r_ref.data_ptr(), ldxf=K, norm=nw.data_ptr(), eps=1e-5)
    hip().bmm(tdw.data_ptr(), int(td), K, F, h_ref.data_ptr(), F, r_ref.data_ptr(), K, B, stream())
    torch.cuda.synchronize()
    _, _, n_ints = hip().chain_layout()
    cnt = torch.zeros(n_ints, dtype=torch.int32, device="cuda")
    for _ in range(3):
        cnt.zero_()
        r = resid0.clone()
        h = torch.full((B, F), 3.0, dtype=torch.float16, device="cuda")
        hip().bmm_wo_ffn_chain(to_.data_ptr(), int(GGMLType.Q4_K), K, dxa.data_ptr(), tg.data_ptr(), int(GGMLType.Q4_K),
                               F, K, nw.data_ptr(), 1e-5, tdw.data_ptr(), int(td), xh.data_ptr(), h.data_ptr(),
                               r.data_ptr(), B, cnt.data_ptr(), stream())
        torch.cuda.synchronize()
        # the SwiGLU rows: equal up to the f16 rounding of inputs whose split-K sums differ in order
        hd = (h.float() - h_ref.float()).abs().max().item()
        assert hd <= 2e-2 * max(1.0, h_ref.float().abs().max().item()), hd
        assert rel_err(r.cpu().numpy() - resid0.cpu().numpy(), r_ref.cpu().numpy() - resid0.cpu().numpy()) < 1e-3


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("B", [1, 6, 8])
@pytest.mark.parametrize("R", [130, 4100])
def test_bmm_store_head_vs_fp32(torch, t, B, R):
    """The batched head's form: f16 rows, one K part, plain stores over whatever the output held
    (the wave-owned kernel's compile-time store epilogue: no zeroed rows to add into), rows past
    n_out untouched."""
    K = 4096
    rng = np.random.default_rng(B * 13 + int(t) + R)
    raw, W = make_matrix(t, R, K, rng)
    dw = dev_bytes(to_planar(t, raw, R, K))
    X = rng.standard_normal((B, K)).astype(np.float32)
    dxh = torch.from_numpy(_swizzle4(X.astype(np.float16))).cuda()
    tw = torch.empty(hip().t16_bytes(int(t), R, K), dtype=torch.uint8, device="cuda")
    hip().t16_repack(dw.data_ptr(), int(t), R, K, tw.data_ptr(), stream(), swiglu=False)
    ldo = R + 6
    out = torch.full((B, ldo), 5.0, device="cuda")
    hip().bmm(tw.data_ptr(), int(t), R, K, dxh.data_ptr(), K, out.data_ptr(), ldo, B, stream(), store_out=True)
    torch.cuda.synchronize()
    pre = X.astype(np.float16).astype(np.float64) @ W.astype(np.float64).T
    got = out.cpu().numpy()
    for b in range(B):
        assert rel_err(got[b, :R], pre[b]) < 3e-3, (b, rel_err(got[b, :R], pre[b]))
        assert np.all(got[b, R:] == 5.0)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("B", [1, 6, 16])
@pytest.mark.parametrize("mode", ["store", "swiglu"])
def test_bmm_folded_norm_vs_fp32(torch, t, B, mode):
    """RMSNorm folded into the one-part staging: fp32 rows in, f16(x * w) staged, the column
    scale rsqrt(mean(x^2) + eps) applied to the reduced tile; `store` writes the result over
    the output, `swiglu` feeds the gate/up epilogue."""
    K = 4096 if B <= 8 else 2048
    if not hip().bmm_norm_fits(K, B):
        pytest.skip("shape outside the folded-norm staging")
    rng = np.random.default_rng(B * 7 + int(t) + (mode == "swiglu"))
    R = 192 if mode == "swiglu" else 130
    raw, W = make_matrix(t, R, K, rng)
    dw = dev_bytes(to_planar(t, raw, R, K))
    X = (rng.standard_normal((B, K)) * 3).astype(np.float32)
    nw = (0.5 + rng.random(K)).astype(np.float32)
    eps = 1e-5
    ldxf = K + 4
    dx = torch.zeros(B, ldxf, device="cuda")
    dx[:, :K] = torch.from_numpy(X).cuda()
    dn = torch.from_numpy(nw).cuda()
    tw = torch.empty(hip().t16_bytes(int(t), R, K), dtype=torch.uint8, device="cuda")
    hip().t16_repack(dw.data_ptr(), int(t), R, K, tw.data_ptr(), stream(), swiglu=(mode == "swiglu"))
    xn = X.astype(np.float64) / np.sqrt((X.astype(np.float64) ** 2).mean(1, keepdims=True) + eps) * nw
    pre = xn @ W.astype(np.float64).T
    if mode == "store":
        ldo = R + 6
        out = torch.full((B, ldo), 5.0, device="cuda")
        hip().bmm(tw.data_ptr(), int(t), R, K, 0, 0, out.data_ptr(), ldo, B, stream(),
                  xf=dx.data_ptr(), ldxf=ldxf, norm=dn.data_ptr(), eps=eps, store_out=True)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for b in range(B):
            assert rel_err(got[b, :R], pre[b]) < 3e-3, (b, rel_err(got[b, :R], pre[b]))
            assert np.all(got[b, R:] == 5.0)
    else:
        F = R // 2
        hout = torch.zeros((B, F), dtype=torch.float16, device="cuda")
        hip().bmm(tw.data_ptr(), int(t), R, K, 0, 0, 0, 0, B, stream(), h_out=hout.data_ptr(), ldh_out=F,
                  xf=dx.data_ptr(), ldxf=ldxf, norm=dn.data_ptr(), eps=eps)
        torch.cuda.synchronize()
        got = hout.cpu().numpy().astype(np.float64)
        g = pre.reshape(B, F // 32, 2, 32)[:, :, 0].reshape(B, F)
        u = pre.reshape(B, F // 32, 2, 32)[:, :, 1].reshape(B, F)
        ref = g / (1.0 + np.exp(-g)) * u
        for b in range(B):
            row = _swizzle4(got[b][None])[0]
            assert rel_err(row, ref[b]) < 3e-3, (b, rel_err(row, ref[b]))


def test_bprep_norm_swiglu_zero(torch):
    """bprep: RMSNorm per row, SwiGLU on interleaved gate/up rows, f16 + (0,2,1,3) swizzle,
    and the zero side job."""
    rng = np.random.default_rng(5)
    B, K = 5, 4096
    X = (rng.standard_normal((B, K)) * 3).astype(np.float32)
    nw = (1 + 0.1 * rng.standard_normal(K)).astype(np.float32)
    dx, dn = torch.from_numpy(X).cuda(), torch.from_numpy(nw).cuda()
    xh = torch.zeros(B, K, dtype=torch.float16, device="cuda")
    z = torch.ones(1024, device="cuda")
    hip().bprep(dx.data_ptr(), K, False, dn.data_ptr(), 1e-5, K, B, xh.data_ptr(), K, stream(), z.data_ptr(), 1024)
    torch.cuda.synchronize()
    want = np.stack([rmsnorm(X[b], nw) for b in range(B)]).astype(np.float16)
    assert rel_err(xh.cpu().numpy().astype(np.float32), _swizzle4(want).astype(np.float32)) < 1e-3
    assert float(z.abs().sum()) == 0.0
    GU = rng.standard_normal((B, 2 * K)).astype(np.float32)
    dgu = torch.from_numpy(GU).cuda()
    for G in (32, 8):   # planar gate / up groups, and the SwiGLU tile16 copy's 8-row groups
        hip().bprep(dgu.data_ptr(), 2 * K, True, 0, 1e-5, K, B, xh.data_ptr(), K, stream(), swiglu_group=G)
        torch.cuda.synchronize()
        g = GU.reshape(B, -1, 2, G)[:, :, 0, :].reshape(B, K)
        u = GU.reshape(B, -1, 2, G)[:, :, 1, :].reshape(B, K)
        h = (g / (1 + np.exp(-g)) * u).astype(np.float16)
        assert rel_err(xh.cpu().numpy().astype(np.float32), _swizzle4(h).astype(np.float32)) < 2e-3, G


@pytest.mark.parametrize("t,T,R,K", [(t, T, R, K) for t in BM_TYPES
                                     for T, R, K in [(17, 256, 512), (100, 4096, 1024), (300, 272, 4096), (130, 1024, 14336)]]
                         + [(GGMLType.Q4_K, 2304, 4096, 512)])   # a joint-admission sized grid
def test_gemm_t16_vs_fp32(torch, t, T, R, K):
    """Prefill GEMM on the tile16 copy: Y = X W^T with X f16 in the 4-group k order and W the
    tile16 dequantisation (f16 arithmetic), against the fp64 product of the same f16 X and the
    exact weights; STORE (split-K on the narrow shapes), STORE + resid, and ADD."""
    rng = np.random.default_rng(T + R + K + int(t))
    raw, W = make_matrix(t, R, K, rng)
    dw = dev_bytes(to_planar(t, raw, R, K))
    tw = torch.empty(hip().t16_bytes(int(t), R, K), dtype=torch.uint8, device="cuda")
    hip().t16_repack(dw.data_ptr(), int(t), R, K, tw.data_ptr(), stream())
    Xh = rng.standard_normal((T, K)).astype(np.float16)
    dx = torch.from_numpy(_swizzle4(Xh)).cuda()
    ref = Xh.astype(np.float64) @ W.astype(np.float64).T
    ldo = R + 4
    out = torch.full((T, ldo), 3.0, device="cuda")
    hip().gemm_t16(tw.data_ptr(), int(t), R, K, dx.data_ptr(), T, out.data_ptr(), ldo, 0, 0, 0, stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert rel_err(got[:, :R], ref) < 2e-3, rel_err(got[:, :R], ref)
    assert np.all(got[:, R:] == 3.0)
    res = torch.randn(T, ldo, device="cuda")
    hip().gemm_t16(tw.data_ptr(), int(t), R, K, dx.data_ptr(), T, out.data_ptr(), ldo, 0, 0, 0, stream(),
                   resid=res.data_ptr())
    torch.cuda.synchronize()
    assert rel_err(out.cpu().numpy()[:, :R] - res.cpu().numpy()[:, :R], ref) < 2e-3
    base = torch.randn(T, ldo, device="cuda")
    acc = base.clone()
    hip().gemm_t16(tw.data_ptr(), int(t), R, K, dx.data_ptr(), T, acc.data_ptr(), ldo, 0, 0, 1, stream())
    torch.cuda.synchronize()
    assert rel_err((acc - base).cpu().numpy()[:, :R], ref) < 2e-3
    assert torch.equal(acc[:, R:], base[:, R:])


@pytest.mark.parametrize("t,T", [(GGMLType.Q4_K, 387), (GGMLType.Q4_K, 17), (GGMLType.Q6_K, 130)])
def test_gemm_t16_stacked_qkv(torch, t, T):
    """Q|K|V in ONE prefill launch (GemmT16Args::wseg_*): three separately repacked tile16 copies
    (4096 / 1024 / 1024 rows) stacked by tile range, their outputs adjacent columns of one [T][ncol]
    buffer, against the fp64 products of each matrix."""
    rng = np.random.default_rng(T + int(t))
    K, rows = 4096, [4096, 1024, 1024]
    Ws, tws = [], []
    for R in rows:
        raw, W = make_matrix(t, R, K, rng)
        dw = dev_bytes(to_planar(t, raw, R, K))
        tw = torch.empty(hip().t16_bytes(int(t), R, K), dtype=torch.uint8, device="cuda")
        hip().t16_repack(dw.data_ptr(), int(t), R, K, tw.data_ptr(), stream())
        Ws.append(W)
        tws.append(tw)
    Xh = rng.standard_normal((T, K)).astype(np.float16)
    dx = torch.from_numpy(_swizzle4(Xh)).cuda()
    ncol = sum(rows)
    ldo = ncol + 4
    out = torch.full((T, ldo), 3.0, device="cuda")
    hip().gemm_t16(tws[0].data_ptr(), int(t), ncol, K, dx.data_ptr(), T, out.data_ptr(), ldo, 0, 0, 0, stream(),
                   wseg=[(tw.data_ptr(), R) for tw, R in zip(tws, rows)])
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    c = 0
    for W, R in zip(Ws, rows):
        ref = Xh.astype(np.float64) @ W.astype(np.float64).T
        assert rel_err(got[:, c:c + R], ref) < 2e-3, (c, rel_err(got[:, c:c + R], ref))
        c += R
    assert np.all(got[:, ncol:] == 3.0)


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
@pytest.mark.parametrize("T,F,K", [(40, 96, 2048), (200, 256, 4096), (129, 1792, 1024),
                                   (330, 512, 1024), (500, 384, 2048), (2050, 256, 512)])  # each block shape
def test_gemm_t16_swiglu_vs_fp32(torch, t, T, F, K):
    """Prefill gate/up on the SwiGLU tile16 copy: silu(gate) * up as f16 in the 4-group k order."""
    rng = np.random.default_rng(T * 3 + F + int(t))
    R = 2 * F
    raw, W = make_matrix(t, R, K, rng)
    dw = dev_bytes(to_planar(t, raw, R, K))
    tw = torch.empty(hip().t16_bytes(int(t), R, K), dtype=torch.uint8, device="cuda")
    hip().t16_repack(dw.data_ptr(), int(t), R, K, tw.data_ptr(), stream(), swiglu=True)
    Xh = rng.standard_normal((T, K)).astype(np.float16)
    dx = torch.from_numpy(_swizzle4(Xh)).cuda()
    ldh = F + 8
    h = torch.full((T, ldh), 7.0, dtype=torch.float16, device="cuda")
    hip().gemm_t16(tw.data_ptr(), int(t), R, K, dx.data_ptr(), T, 0, 0, h.data_ptr(), ldh, 2, stream())
    torch.cuda.synchronize()
    pre = Xh.astype(np.float64) @ W.astype(np.float64).T
    g = pre.reshape(T, F // 32, 2, 32)[:, :, 0].reshape(T, F)
    u = pre.reshape(T, F // 32, 2, 32)[:, :, 1].reshape(T, F)
    ref = g / (1.0 + np.exp(-g)) * u
    got = h.cpu().numpy().astype(np.float64)
    assert rel_err(_swizzle4(got[:, :F]), ref) < 3e-3, rel_err(_swizzle4(got[:, :F]), ref)
    assert np.all(got[:, F:] == 7.0)


def test_rmsnorm_f16_swizzled(torch):
    rng = np.random.default_rng(5)
    T, d = 7, 4096
    x = torch.from_numpy((rng.standard_normal((T, d)) * 2).astype(np.float32)).cuda()
    w = torch.from_numpy((0.5 + rng.random(d)).astype(np.float32)).cuda()
    y = torch.zeros(T, d, dtype=torch.float16, device="cuda")
    hip().rmsnorm_bf16(x.data_ptr(), w.data_ptr(), 1e-5, T, d, y.data_ptr(), stream(), f16sw=True)
    torch.cuda.synchronize()
    xf = x.cpu().double()
    ref = (xf / torch.sqrt((xf * xf).mean(1, keepdim=True) + 1e-5) * w.cpu().double()).numpy()
    assert rel_err(_swizzle4(y.float().cpu().numpy()), ref) < 1e-3


def _rope_table(n_ctx, hd, theta=5e5):
    inv = theta ** (-np.arange(0, hd, 2, dtype=np.float64) / hd)
    ang = np.arange(n_ctx, dtype=np.float64)[:, None] * inv[None, :]
    return np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32)   # [n_ctx][hd/2][2]


def _rope_pairs(y, pos, tab):
    """RoPE on adjacent pairs (GGUF normal mode) of y [rows] at position pos, rows % hd per head."""
    hd2 = tab.shape[1]
    z = y.reshape(-1, hd2, 2).astype(np.float64)
    c, s = tab[pos, :, 0].astype(np.float64), tab[pos, :, 1].astype(np.float64)
    return np.stack([z[..., 0] * c - z[..., 1] * s, z[..., 0] * s + z[..., 1] * c], -1).reshape(y.shape)


@pytest.mark.parametrize("types", [(GGMLType.Q4_K,) * 3, (GGMLType.Q4_K, GGMLType.Q4_K, GGMLType.Q6_K),
                                   (GGMLType.Q4_K, GGMLType.Q8_0, GGMLType.Q8_0)])
@pytest.mark.parametrize("B", [1, 6, 8])
@pytest.mark.parametrize("hd,H,Hkv,K", [(128, 32, 8, 4096), (64, 32, 4, 2048)])
def test_bmm_qkv_splitk_then_attention(torch, types, B, hd, H, Hkv, K):
    """Split-K Q|K|V (RoPE'd partial sums of f16(x * norm_w) . W, the rows' sums of squares) and the
    batched attention that normalises them, appends the new K / V at each row's position and
    attends over the cache + the new key - against fp64 references of both stages."""
    tq, tk, tv = types
    if not hip().bmm_qkv_sk_supported(int(tq), int(tk), int(tv), K, B):
        pytest.skip("type mix outside the split-K launch")
    rng = np.random.default_rng(B * 31 + hd + int(tv) + int(tk))
    n_ctx, nq, nkv = 256, H * hd, Hkv * hd
    mats = []
    for t, R in ((tq, nq), (tk, nkv), (tv, nkv)):
        raw, W = make_matrix(t, R, K, rng)
        dw = dev_bytes(to_planar(t, raw, R, K))
        tw = torch.empty(hip().t16_bytes(int(t), R, K), dtype=torch.uint8, device="cuda")
        hip().t16_repack(dw.data_ptr(), int(t), R, K, tw.data_ptr(), stream())
        mats.append((tw, W, dw))
    X = (rng.standard_normal((B, K)) * 3).astype(np.float32)
    nw = (0.5 + rng.random(K)).astype(np.float32)
    eps = 1e-5
    tab = _rope_table(n_ctx, hd)
    pos = rng.integers(1, n_ctx, B).astype(np.int32)
    slots = rng.permutation(8)[:B].astype(np.int32)
    ldo = nq + 2 * nkv
    dx, dn = torch.from_numpy(X).cuda(), torch.from_numpy(nw).cuda()
    dtab, dpos, dslots = torch.from_numpy(tab).cuda(), torch.from_numpy(pos).cuda(), torch.from_numpy(slots).cuda()
    dfreq = torch.from_numpy((5e5 ** (-np.arange(0, hd, 2, dtype=np.float64) / hd)).astype(np.float32)).cuda()
    out = torch.zeros(B, ldo, device="cuda")
    ss = torch.zeros(16, device="cuda")
    hip().bmm_qkv_sk(mats[0][0].data_ptr(), int(tq), nq, mats[1][0].data_ptr(), int(tk), mats[2][0].data_ptr(), int(tv),
                     nkv, K, dx.data_ptr(), K, dn.data_ptr(), eps, B, out.data_ptr(), ldo, ss.data_ptr(),
                     dpos.data_ptr(), dtab.data_ptr(), hd, n_ctx, stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy().astype(np.float64)
    xw = (X * nw).astype(np.float16).astype(np.float64)
    ss_ref = (X.astype(np.float64) ** 2).sum(1)
    assert np.allclose(ss.cpu().numpy()[:B], ss_ref, rtol=1e-5)
    raw_ref = []
    # the interleaved-step kernels leave the sums un-RoPE'd; the attention then rotates q / the new key
    deferred = hip().bmm_qkv_sk_defers_rope()
    for b in range(B):
        q = _rope_pairs(xw[b] @ mats[0][1].astype(np.float64).T, pos[b], tab)
        k = _rope_pairs(xw[b] @ mats[1][1].astype(np.float64).T, pos[b], tab)
        v = xw[b] @ mats[2][1].astype(np.float64).T
        qg, kg = got[b, :nq], got[b, nq:nq + nkv]
        if deferred:
            qg, kg = _rope_pairs(qg, pos[b], tab), _rope_pairs(kg, pos[b], tab)
        for name, g, r in (("q", qg, q), ("k", kg, k), ("v", got[b, nq + nkv:], v)):
            assert rel_err(g, r) < 3e-3, (b, name, rel_err(g, r))
        raw_ref.append((q, k, v))
    # stage 2: the batched attention over the raw sums
    slot_stride = Hkv * n_ctx * hd
    Kc = rng.standard_normal((8, Hkv, n_ctx, hd)).astype(np.float16)
    Vc = rng.standard_normal((8, Hkv, n_ctx, hd)).astype(np.float16)
    dK, dV = torch.from_numpy(Kc).cuda(), torch.from_numpy(Vc).cuda()
    part = torch.zeros(B * hip().attn_decode_workspace_floats(n_ctx, H, hd), device="cuda")
    cnt = torch.zeros(64 * B, dtype=torch.int32, device="cuda")
    aout = torch.zeros(B, nq, device="cuda")
    aouth = torch.zeros(B, nq, dtype=torch.float16, device="cuda")
    scale = 1 / np.sqrt(hd)
    hip().attn_decode(out.data_ptr(), dK.data_ptr(), dV.data_ptr(), dpos.data_ptr(), n_ctx, H, Hkv, hd, scale,
                      part.data_ptr(), aout.data_ptr(), stream(), cnt.data_ptr(), batch=B, slots=dslots.data_ptr(),
                      slot_stride=slot_stride, out_h=aouth.data_ptr(), qkv_raw=out.data_ptr(), qkv_ld=ldo, k_off=nq,
                      v_off=nq + nkv, ss=ss.data_ptr(), inv_k=1.0 / K, eps=eps,
                      rope_freq=dfreq.data_ptr() if deferred else 0)
    torch.cuda.synchronize()
    Kg, Vg, ao = dK.cpu().numpy(), dV.cpu().numpy(), aout.cpu().numpy()
    for b in range(B):
        q, k, v = raw_ref[b]
        rs = 1.0 / np.sqrt(ss_ref[b] / K + eps)
        kn = (k * rs).astype(np.float16).reshape(Hkv, hd)
        vn = (v * rs).astype(np.float16).reshape(Hkv, hd)
        s, p = slots[b], pos[b]
        assert rel_err(Kg[s, :, p].astype(np.float64), kn.astype(np.float64)) < 3e-3
        assert rel_err(Vg[s, :, p].astype(np.float64), vn.astype(np.float64)) < 3e-3
        Kr, Vr = Kc[s].copy(), Vc[s].copy()
        Kr[:, p], Vr[:, p] = kn, vn
        ref = _attn_ref((q * rs).reshape(H, hd), Kr, Vr, p + 1, scale)
        assert rel_err(ao[b].reshape(H, hd), ref) < 5e-3, (b, rel_err(ao[b].reshape(H, hd), ref))
        # rows of the other slots' caches untouched
    untouched = [s for s in range(8) if s not in set(slots.tolist())]
    for s in untouched:
        assert np.array_equal(Kg[s], Kc[s]) and np.array_equal(Vg[s], Vc[s])
    assert int(cnt.abs().sum()) == 0
