"""The engine's RCCL branch, exercised on the one-GPU test box.

RCCL refuses two ranks on one device, so the multi-rank GPU tests run their collectives on
the P2P kernel (comm="ipc"). Here ``comm="rccl"`` at tp_size 1 runs every tensor-parallel
code path of the engine over a ONE-rank RCCL communicator created by the engine itself
(ncclCommInitRank): the row-parallel all-reduces of prefill, graph-captured decode and the
batched step, and the vocabulary-parallel sampler's candidate all-gather - each an
ncclAllReduce / ncclAllGather enqueued on the engine stream, captured into its hipGraphs and
replayed step after step. A one-rank all-reduce is a copy, so the results must match the
plain engine's to its own run-to-run noise (split-K float atomics)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


@pytest.mark.timeout(300)
def test_rccl_one_rank_engine_matches_plain(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    path = write_synthetic_gguf("tiny-llama3-q4_k_m", str(tmp_path / "m.gguf"), seed=2)
    kw = dict(n_ctx=256, n_batch=64, device=0, use_graph=True, n_slots=4)
    plain = hip.Engine(path, **kw)
    rccl = hip.Engine(path, tp_rank=0, tp_size=1, nccl_id=hip.nccl_unique_id(), comm="rccl", **kw)
    toks = [int(t) for t in np.random.default_rng(5).integers(3, 400, 60)]
    # prefill: T x d all-reduces (RCCL) after Wo / down of every layer
    assert _rel(rccl.eval_logits(toks[:50], 0), plain.eval_logits(toks[:50], 0)) < 2e-3
    # graph-replayed decode steps (two all-reduces per layer + the sampler's candidate all-gather)
    for i in range(4):
        assert _rel(rccl.decode_logits(toks[50 + i], 50 + i), plain.decode_logits(toks[50 + i], 50 + i)) < 2e-3
    g1 = rccl.generate(toks[:20], 0, 24, {"temperature": 0.0}, [], None, None)["tokens"]
    g0 = plain.generate(toks[:20], 0, 24, {"temperature": 0.0}, [], None, None)["tokens"]
    assert g1[:12] == g0[:12], (g1, g0)
    # batched steps: one captured graph per row count, replayed with RCCL collectives inside
    sp = {"temperature": 0.0}
    prompts = [toks[3 * i:3 * i + 9] for i in range(3)]
    outs = []
    for eng in (rccl, plain):
        eng.slots_begin([1, 2, 3], prompts, [0, 0, 0], [sp] * 3)
        outs.append([eng.batch_step([1, 2, 3]) for _ in range(10)])
    assert outs[0][:6] == outs[1][:6], outs
    assert rccl.healthy and plain.healthy
