"""The row-parallel decode GEMV's epilogue all-reduce (gemv.hip tp_store_row, GemvArgs::tp_*) at
the group sizes BASELINE's TP configs use (2, 4 and 8 ranks), in ONE process on one GPU.

Only rank R's launch runs; its W - 1 peers are simulated by pre-writing their {value, epoch}
granules into rank R's region (parity epoch & 1, slot (parity, peer), the fused-area offset), as
their launches would have. That exercises exactly the code a TP = 8 node runs - the per-row
epoch, the parity flip over consecutive launches, the push of rank R's own row to every region,
the rank-order sum and the residual - without eight co-scheduled processes. The poison path: a
fault word raised by some rank ends the wait at once and leaves the rows unwritten."""
import time

import numpy as np
import pytest

from llama_fastapi_k8s_gpu_amd.gguf.constants import GGMLType
from gpu_helpers import dev_bytes, hip, make_matrix, q8_emulate, rel_err, stream, to_planar

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def granules(epoch, vals):
    """{value, epoch} 8-byte granules as the kernels write them (epoch in the high word)."""
    v = np.asarray(vals, np.float32).view(np.uint32).astype(np.uint64)
    return ((np.uint64(epoch) << np.uint64(32)) | v).view(np.int64)


@pytest.mark.parametrize("W,rank", [(2, 1), (4, 0), (4, 3), (8, 5), (8, 7)])
def test_epilogue_allreduce_group(torch, W, rank):
    rng = np.random.default_rng(100 * W + rank)
    t, R, K = GGMLType.Q4_K, 8192, 1024          # the 70B Wo slice of one rank at TP = 8
    raw, Wm = make_matrix(t, R, K, rng)
    dw = dev_bytes(to_planar(t, raw, R, K))
    x = rng.standard_normal(K).astype(np.float32)
    dx = torch.from_numpy(x).cuda()
    own_ref = Wm.astype(np.float64) @ q8_emulate(x).astype(np.float64)
    off = 96                                       # the fused area sits past the collective's granules
    stride = off + R
    regions = [torch.zeros(2 * W * stride, dtype=torch.int64, device="cuda") for _ in range(W)]
    faults = [torch.zeros(8, dtype=torch.int32, device="cuda") for _ in range(W)]
    epochs = torch.zeros(R, dtype=torch.int32, device="cuda")
    err = torch.zeros(4, dtype=torch.int32, device="cuda")
    data_ptrs = [r.data_ptr() for r in regions]
    fault_ptrs = [f.data_ptr() for f in faults]
    h = hip()
    for e in (1, 2, 3):                            # parity 1, 0, 1: the slots alternate per launch
        par = e & 1
        peer = {p: rng.standard_normal(R).astype(np.float32) for p in range(W) if p != rank}
        mine = regions[rank]
        for p, v in peer.items():                  # the peers' pushes into rank R's region
            a = (par * W + p) * stride + off
            mine[a:a + R] = torch.from_numpy(granules(e, v)).cuda()
        resid = rng.standard_normal(R).astype(np.float32)
        dres = torch.from_numpy(resid).cuda()
        out = torch.full((R,), float("nan"), device="cuda")
        h.gemv_tp(dw.data_ptr(), int(t), R, K, dx.data_ptr(), out.data_ptr(), R, dres.data_ptr(), data_ptrs,
                  fault_ptrs, rank, stride, off, epochs.data_ptr(), err.data_ptr(), stream())
        torch.cuda.synchronize()
        # rank R's own row went to every region (its own included), tagged with this launch's epoch
        pushed = []
        for p in range(W):
            a = (par * W + rank) * stride + off
            g = regions[p][a:a + R].cpu().numpy().view(np.uint64)
            assert np.all((g >> np.uint64(32)) == e), (p, e)
            pushed.append((g & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32))
        own = pushed[rank]
        assert all(np.array_equal(own, q) for q in pushed)
        assert rel_err(own, own_ref) < 2e-4
        # out = resid + the rank-order fp32 sum, bit for bit
        acc = np.zeros(R, np.float32)
        for p in range(W):
            acc = acc + (own if p == rank else peer[p])
        want = resid + acc
        got = out.cpu().numpy()
        assert np.array_equal(got, want), (e, float(np.abs(got - want).max()))
        assert int(err.cpu().numpy()[0]) == 0
    assert np.all(epochs.cpu().numpy() == 3)
    # poison: one peer's granules never arrive, but some rank raised its fault word - the wait ends
    # at once (not after its 20 s bound), no row is written, no new fault is raised by this rank
    q = (rank + 1) % W
    faults[rank][q] = 300 + q
    e, par = 4, 0
    for p in range(W):
        if p not in (rank, q):
            a = (par * W + p) * stride + off
            regions[rank][a:a + R] = torch.from_numpy(granules(e, np.ones(R, np.float32))).cuda()
    out = torch.full((R,), float("nan"), device="cuda")
    t0 = time.time()
    h.gemv_tp(dw.data_ptr(), int(t), R, K, dx.data_ptr(), out.data_ptr(), R, 0, data_ptrs, fault_ptrs, rank, stride,
              off, epochs.data_ptr(), err.data_ptr(), stream())
    torch.cuda.synchronize()
    assert time.time() - t0 < 5.0
    assert np.isnan(out.cpu().numpy()).all()
    assert int(err.cpu().numpy()[0]) == 0
    assert faults[rank].cpu().numpy()[rank] == 0
