"""One-shot P2P all-reduce / all-gather (kernels/p2p_allreduce.hip, runtime/p2p.cpp).

Two processes share the ONE GPU of the test box: each exports its receive region
with a hipIpc handle, the handles are exchanged over a gloo group, and the
all-reduce runs exactly as on an 8-GPU node, minus the xGMI transport (the
peer pointer is an IPC mapping of the same device's memory). Checked against
the fp32 sum in rank order, over many epochs (slot reuse) and under hipGraph
replay (epochs advance on the device)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 4096


def _inputs(rank, it, n=N):
    return np.random.default_rng(1000 * it + rank).standard_normal(n).astype(np.float32)


def _worker(rank, world, port, q, uncached):
    try:
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from llama_fastapi_k8s_gpu_amd.parallel.comm import allgather_bytes
        from llama_fastapi_k8s_gpu_amd.runtime import load_hip
        hip = load_hip()
        c = hip.P2PComm(rank, world, N, 0, uncached=uncached)
        if uncached:
            assert c.uncached, "hipDeviceMallocUncached refused"
        # device memory freed and re-allocated between the region's setup and the first
        # collective (the engine's MoE setup does this): the region is a whole allocation of its
        # own (runtime/p2p.cpp checks it), so nothing carved out of the freed blocks aliases it
        junk = [torch.empty(3 << 20, dtype=torch.uint8, device="cuda") for _ in range(4)]
        del junk
        torch.cuda.empty_cache()
        junk2 = torch.full((5 << 20,), 7, dtype=torch.uint8, device="cuda")  # noqa: F841
        c.open(allgather_bytes(c.handle()))
        s = torch.cuda.current_stream()
        src = torch.empty(N, device="cuda")
        dst = torch.empty(N, device="cuda")
        worst = 0.0
        for it in range(40):   # eager: 40 epochs, both slots reused 20 times
            n = N if it % 3 else 1000 + it
            src[:n].copy_(torch.from_numpy(_inputs(rank, it, n)))
            dist.barrier()
            c.allreduce(src.data_ptr(), dst.data_ptr(), n, s.cuda_stream)
            torch.cuda.synchronize()
            ref = sum(_inputs(r, it, n).astype(np.float32) for r in range(world))
            worst = max(worst, float(np.abs(dst[:n].cpu().numpy() - ref).max()))
        # back-to-back launches of different sizes with no host barrier in between (the fixed
        # grid keeps slot reuse safe), all-gathers interleaved with all-reduces
        outs = []
        for it in range(12):
            n = [N, 37, 1000 + it][it % 3]
            x = torch.from_numpy(_inputs(rank, 200 + it, n)).cuda()
            if it % 2:
                y = torch.empty(n, device="cuda")
                c.allreduce(x.data_ptr(), y.data_ptr(), n, s.cuda_stream)
            else:
                y = torch.empty(world * n, device="cuda")
                c.allgather(x.data_ptr(), y.data_ptr(), n, s.cuda_stream)
            outs.append((it, n, y))
        torch.cuda.synchronize()
        for it, n, y in outs:
            parts = [_inputs(r, 200 + it, n) for r in range(world)]
            ref = sum(parts) if it % 2 else np.concatenate(parts)
            worst = max(worst, float(np.abs(y.cpu().numpy() - ref).max()))
        # accumulating mode (the batched row-parallel projections): dst += sum, src left zeroed
        base = torch.from_numpy(_inputs(7, 500)).cuda()   # the same "residual" on both ranks
        acc = base.clone()
        ref = _inputs(7, 500).astype(np.float32)
        for it in range(4):
            n = [N, 1000, 37, N][it]
            src.zero_()
            src[:n].copy_(torch.from_numpy(_inputs(rank, 600 + it, n)))
            dist.barrier()
            c.allreduce_add(src.data_ptr(), acc.data_ptr(), n, s.cuda_stream)
            torch.cuda.synchronize()
            ref[:n] += sum(_inputs(r, 600 + it, n) for r in range(world))
            assert float(src.abs().max()) == 0.0, "accumulate: src not zeroed"
            worst = max(worst, float(np.abs(acc.cpu().numpy() - ref).max()))
        # graph replay: the captured launch advances its epochs on the device
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        src.copy_(torch.from_numpy(_inputs(rank, 99)))
        with torch.cuda.stream(cs):
            with torch.cuda.graph(g):
                c.allreduce(src.data_ptr(), dst.data_ptr(), N, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ref = sum(_inputs(r, 99) for r in range(world))
        for _ in range(10):
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            worst = max(worst, float(np.abs(dst.cpu().numpy() - ref).max()))
        q.put((rank, worst, c.error(), dst[:8].cpu().numpy().tolist()))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, repr(e), None))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("uncached", [True, False])
def test_p2p_allreduce_two_processes_one_gpu(uncached):
    """Both region types: hipDeviceMallocUncached (the engine's) and plain hipMalloc; device memory
    is freed and re-allocated between the regions' setup and the handle exchange."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port + (0 if uncached else 7), q, uncached)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort()
    for rank, worst, err, head in res:
        assert worst is not None, err
        assert err == 0, f"rank {rank}: device error word {err}"
        assert worst < 1e-5, (rank, worst)
    assert res[0][3] == res[1][3]   # bit-identical on both ranks


def test_p2p_uncached_region_one_rank():
    """One rank on an uncached region (no IPC import at all): the collective's own stores,
    flags and system-scope loads, eager and graph-replayed."""
    import torch
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    c = hip.P2PComm(0, 1, N, 0, uncached=True)
    if not c.uncached:
        pytest.skip("hipDeviceMallocUncached refused on this device")
    c.open([b"self"])
    s = torch.cuda.current_stream()
    for it in range(6):
        n = [N, 37, 1000][it % 3]
        x = torch.from_numpy(_inputs(0, 300 + it, n)).cuda()
        y = torch.empty(n, device="cuda")
        c.allreduce(x.data_ptr(), y.data_ptr(), n, s.cuda_stream)
        z = torch.empty(n, device="cuda")
        c.allgather(x.data_ptr(), z.data_ptr(), n, s.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(y, x) and torch.equal(z, x)
        xs = x.clone()
        y0 = y.clone()
        c.allreduce_add(xs.data_ptr(), y.data_ptr(), n, s.cuda_stream)   # one rank: y += x, x zeroed
        torch.cuda.synchronize()
        assert torch.equal(y, y0 + x) and float(xs.abs().max()) == 0.0
    x = torch.from_numpy(_inputs(0, 400, N)).cuda()
    y = torch.zeros(N, device="cuda")
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        with torch.cuda.graph(g):
            c.allreduce(x.data_ptr(), y.data_ptr(), N, torch.cuda.current_stream().cuda_stream)
    for k in range(3):
        x.add_(1.0)
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, x)
    assert c.error() == 0
