"""Tensor parallelism at TP = 8 on the 70B layer shape (BASELINE config 4), rehearsed on one GPU.

Eight ranks share device 0 over the IPC comm mode (as tests/test_tp_gpu.py does for two) and
serve a 2-layer model of Llama-3-70B's width: d = 8192, 64 query / 8 KV heads, F = 28672, so
every rank holds the exact per-rank shapes of a 70B TP = 8 deployment - ONE KV head, 8 query
heads and F_l = 3584 FFN features per rank, a 1/8 vocabulary shard - and its all-reduces carry
the 70B's 8192-wide rows. Rank 0 drives, ranks 1-7 replay its commands over the native control
channel.

Checked against the same model at TP = 1 (rank 0, after the group closed) and the exact fp32
model (ReferenceLlama on the GPU): prefill logits within 5e-3 of TP = 1; graph-replayed decode
logits within 2e-2 of TP = 1 and no further from the exact model than TP = 1 is (+5e-3) - the
decode steps read the K/V the bf16 / f16 prefill wrote, and eight-way sharded sums over
8192-wide rows flip more of those roundings than test_tp_gpu.py's two-way ones (measured
1.1-1.4 % vs TP = 1, r4); greedy generations identical or diverging at a near-tie of the TP = 1
logits, two rows of continuous batching identical or diverging at a near-tie of the exact model,
every rank healthy.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD = 8
SPEC = "llama3-70b-2l"


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def _exercise(llm):
    eng = llm._backend.engine
    toks = [int(t) for t in np.random.default_rng(7).integers(3, 400, 28)]
    out = {"prefill": eng.eval_logits(toks[:24], 0)}
    out["decode"] = [eng.decode_logits(toks[24 + i], 24 + i) for i in range(3)]
    out["greedy"] = eng.generate(toks[:12], 0, 16, {"temperature": 0.0}, [], None, None)["tokens"]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(2) as ex:
        res = list(ex.map(lambda i: llm.create_completion([1, 7 + i, 11, 19 + i], max_tokens=8, temperature=0.0),
                          range(2)))
    out["batched"] = [x["choices"][0]["text"] for x in res]
    out["batched_tokens"] = [llm.tokenize(t.encode(), add_bos=False, special=True) for t in out["batched"]]
    out["healthy"] = bool(llm.health()["ok"])
    return out


def _worker(rank, world, port, path, q):
    try:
        # one hardware queue per process: eight processes x the default four oversubscribe the
        # queue scheduler, which then time-slices them (tools/p2p_latency.py, r4)
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK="0")
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
        kw = dict(n_gpu_layers=-1, n_ctx=128, n_batch=64, seed=5, verbose=False, max_batch=2)
        llm = Llama(path, split_mode="row", tp_comm="ipc", device=0, **kw)
        assert llm._backend.tp_size == world
        result = None
        if rank > 0:
            llm.follow()
            llm.close()
        else:
            got = _exercise(llm)
            llm.close()
            ref_llm = Llama(path, split_mode="none", **kw)
            ref = _exercise(ref_llm)
            # the TP = 1 logits along the TP = 1 greedy path (near-tie judgement)
            toks = [int(t) for t in np.random.default_rng(7).integers(3, 400, 28)][:12]
            k = next((i for i, (x, y) in enumerate(zip(got["greedy"], ref["greedy"])) if x != y), None)
            tie = None
            if k is not None:
                lg = ref_llm._backend.engine.eval_logits(toks + ref["greedy"][:k], 0)
                tie = float(abs(lg[got["greedy"][k]] - lg[ref["greedy"][k]]) / np.abs(lg).max())
            ref_llm.close()
            # the exact fp32 model on the GPU (1.7 G parameters dequantised once)
            import torch
            from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
            from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
            ex = ReferenceLlama(GGUFReader(path), n_ctx=128, device="cuda")
            allt = [int(t) for t in np.random.default_rng(7).integers(3, 400, 28)]
            with torch.no_grad():
                exact = [ex.forward(allt[:24], 0).cpu().numpy()]
                exact += [ex.forward([allt[24 + i]], 24 + i).cpu().numpy() for i in range(3)]
                # a batched row whose greedy text differs: the exact model's margin between the two
                # engines' tokens at the first difference (near-tie judgement, as test_tp_gpu.py)
                bties = []
                for i, (ta, tb) in enumerate(zip(got["batched_tokens"], ref["batched_tokens"])):
                    j = next((n for n, (x, y) in enumerate(zip(ta, tb)) if x != y), None)
                    if got["batched"][i] == ref["batched"][i] or j is None:
                        bties.append(None)
                        continue
                    lg = ex.forward([1, 7 + i, 11, 19 + i] + list(tb[:j]), 0).cpu().numpy()
                    bties.append(float(abs(lg[ta[j]] - lg[tb[j]]) / np.abs(lg).max()))
            del ex
            got["batched_ties"] = bties
            result = (got, ref, k, tie, exact)
        dist.barrier()
        q.put((rank, result, None))
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.timeout(900)
def test_tensor_parallel_eight_ranks_70b_width(tmp_path):
    import torch
    # (device_count does not initialise HIP in this process: no queues held beside the ranks')
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    import torch.multiprocessing as mp

    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    path = write_synthetic_gguf(SPEC, str(tmp_path / f"{SPEC}.gguf"), seed=4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, path, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, result, err = q.get(timeout=840)
            res[rank] = (result, err)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank in range(WORLD):
        assert res[rank][1] is None, f"rank {rank}:\n{res[rank][1]}"
    got, ref, k, tie, exact = res[0][0]
    d = [_rel(got["prefill"], ref["prefill"])] + [_rel(a, b) for a, b in zip(got["decode"], ref["decode"])]
    e_tp = [_rel(a, x) for a, x in zip([got["prefill"]] + got["decode"], exact)]
    e_1 = [_rel(a, x) for a, x in zip([ref["prefill"]] + ref["decode"], exact)]
    report = {"vs_tp1": [round(v, 5) for v in d], "err_tp": [round(v, 5) for v in e_tp],
              "err_tp1": [round(v, 5) for v in e_1], "greedy_diverge_at": k, "tie": tie,
              "batched_same": [a == b for a, b in zip(got["batched"], ref["batched"])],
              "batched_ties": got["batched_ties"]}
    assert d[0] <= 5e-3 and max(d[1:]) <= 2e-2, report
    assert all(t <= o + 5e-3 for t, o in zip(e_tp, e_1)), report
    # a near-tie is one within the rounding noise this run measured: twice the larger logit error
    # of TP = 8 or TP = 1 against the exact model (capped at the old fixed 2e-2)
    noise = min(2e-2, 2.0 * max(e_tp + e_1))
    report["noise"] = round(noise, 5)
    assert k is None or tie <= noise, report
    # continuous batching under TP = 8: every row's text equal, or diverging at a near-tie of the
    # exact model (eight-way sharded sums move the batched rows' logits ~1 %, measured r4)
    assert all(a == b or (t is not None and t <= noise)
               for a, b, t in zip(got["batched"], ref["batched"], got["batched_ties"])), report
    assert got["healthy"], report
    print("TP8 report:", report)
