"""split_mode=LAYER across stages (runtime/layer_split_backend.py) on the GPU: three HIP engines
over layer ranges [0, 2), [2, 3), [3, 4) of a 4-layer model (tensor_split 1:1:2, llama.cpp's
l / (n_layer + 1) rule), rehearsed on device 0 (one GPU box;
on a node each stage sits on its own GPU), against the whole model in one engine. The stages run
the same kernels on the same fp32 hidden states, so the prompt logits agree to rounding of the
identical path (tight), and greedy generation matches the single engine's eval path token by
token (each generated token is the argmax of the whole model's logits for its prefix, or within a
near-tie of it)."""
import numpy as np
import pytest

from gpu_helpers import rel_err
from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def path(tmp_path_factory):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return write_synthetic_gguf("tiny-llama3-q4_k_m", str(tmp_path_factory.mktemp("ls") / "m.gguf"), seed=9)


def test_layer_split_matches_whole_model(path):
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    from llama_fastapi_k8s_gpu_amd.engine.sampling import SamplingParams
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    kw = dict(n_gpu_layers=-1, n_ctx=128, n_batch=32, seed=1, verbose=False)
    split = Llama(path, split_mode="layer", tensor_split=[1, 1, 2], layer_devices=[0, 0, 0], **kw)
    be = split._backend
    assert split.backend_name == "layer"
    assert [(s.layer_begin, s.layer_end, s.has_head) for s in be.stages] == [(0, 2, False), (2, 3, False), (3, 4, True)]
    whole = load_hip().Engine(path, n_ctx=128, n_batch=32, device=0, use_graph=False)
    # each stage holds the KV of its own layers only, and only the first one the embedding
    assert [s.kv_state_bytes(10) for s in be.stages] == [whole.kv_state_bytes(10) * n // 4 for n in (2, 1, 1)]
    assert be.stages[1].device_bytes < be.stages[0].device_bytes
    toks = [int(t) for t in np.random.default_rng(4).integers(3, 400, 40)]
    # a 40-token prompt: chunks of 32 + 8 tokens through all three stages
    got = be.eval_logits(toks, 0)
    whole.eval_logits(toks[:32], 0)
    ref = whole.eval_logits(toks[32:], 32)
    assert rel_err(got, ref) < 1e-4, rel_err(got, ref)
    # the host hand-off (eval_stage with hidden states in / out) gives the same logits
    h0 = be.stages[0].eval_stage(None, toks[32:], 32)
    h1 = be.stages[1].eval_stage(h0, [], 32)
    assert rel_err(be.stages[2].eval_stage(h1, [], 32), ref) < 1e-4
    # a stage without the head returns hidden states [T, d]; it refuses the logits entry points
    h = be.stages[0].eval_stage(None, toks[:5], 0)
    assert h.shape == (5, split.hparams.n_embd) and np.isfinite(h).all()
    with pytest.raises(RuntimeError):
        be.stages[0].eval_logits(toks[:5], 0)
    # greedy generation through the stages (native chain: graphs per stage, device sampler), each
    # token checked against the whole model's prompt-path logits (the decode path quantises its
    # GEMV inputs: a near-tie may go either way)
    prompt = toks[:12]
    assert be.native_chain(SamplingParams(temperature=0.0))
    r = be.generate(prompt, 0, 10, SamplingParams(temperature=0.0), [])
    assert len(r.tokens) == 10
    for i, t in enumerate(r.tokens):
        lg = whole.eval_logits(prompt + r.tokens[:i], 0)
        best = int(np.argmax(lg))
        assert t == best or (lg[best] - lg[t]) <= 2e-2 * np.abs(lg).max(), (i, t, best)
    # the facade path (chat-free completion) runs on the stages too
    out = split.create_completion(prompt, max_tokens=4, temperature=0.0)
    assert out["usage"]["completion_tokens"] >= 1
    assert split.health()["ok"]


def test_layer_split_chain_equals_single_engine_generate(path):
    """The native stage chain (Engine::chain_generate: per-stage decode graphs, hidden rows peer to
    peer, the last stage's device sampler, state copied back to every stage) runs the single
    engine's kernels in the same order on the same values, so its tokens equal the one-engine
    generate's - greedy and seeded sampling alike - and a stop token ends both at the same step."""
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    whole = hip.Engine(path, n_ctx=128, n_batch=32, device=0, use_graph=True)
    be = Llama(path, split_mode="layer", tensor_split=[1, 1, 2], layer_devices=[0, 0, 0], n_gpu_layers=-1,
               n_ctx=128, n_batch=32, seed=1, verbose=False)._backend
    prompt = [int(t) for t in np.random.default_rng(7).integers(3, 400, 45)]  # two prefill chunks
    for sp in ({"temperature": 0.0}, {"temperature": 0.9, "top_k": 40, "top_p": 0.95, "seed": 1234,
                                      "repeat_penalty": 1.1}):
        ref = whole.generate(prompt, 0, 24, sp, [])
        got = hip.chain_generate(be.stages, prompt, 0, 24, sp, [])
        assert got["tokens"] == ref["tokens"], (sp, got["tokens"], ref["tokens"])
        assert got["finish"] == ref["finish"] == "length"
        assert got["n_evaluated"] == ref["n_evaluated"]
    stop = ref["tokens"][5]
    a = whole.generate(prompt, 0, 24, sp, [stop])
    b = hip.chain_generate(be.stages, prompt, 0, 24, sp, [stop])
    assert a["tokens"] == b["tokens"] and b["finish"] == "stop"
    # a chain must cover the layers in order and end at the head
    with pytest.raises(RuntimeError):
        hip.chain_generate(be.stages[1:], prompt, 0, 4, sp, [])
    with pytest.raises(RuntimeError):
        hip.chain_generate(be.stages[:2], prompt, 0, 4, sp, [])
