"""T4/T5/T7 on the GPU: the full MI355X engine on tiny synthetic GGUFs against the
float32 torch reference model; graph vs eager decode; facade generation."""
import numpy as np
import pytest

from gpu_helpers import rel_err
from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf

pytestmark = pytest.mark.gpu

SPECS = ["tiny-llama3-q4_k_m", "tiny-llama3-mixed", "tiny-tinyllama-q8_0", "tiny-mixtral-q4_k_m", "tiny-llama3-f32",
         "tiny-llama3-wide", "tiny-q8-oddff"]


@pytest.fixture(scope="module")
def models(tmp_path_factory):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = tmp_path_factory.mktemp("models")
    return {s: write_synthetic_gguf(s, str(d / f"{s}.gguf"), seed=3) for s in SPECS}


def _engine(path, n_ctx=256, graph=True):
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    return load_hip().Engine(path, n_ctx=n_ctx, n_batch=128, device=0, use_graph=graph)


@pytest.mark.parametrize("spec", SPECS)
def test_prefill_and_decode_logits_match_reference(models, spec):
    """Prefill (MFMA GEMM) and decode (GEMV) logits against the fp32 model that reproduces
    each path's rounding (ReferenceLlama path=...): tight; and against the exact model: the
    rounding's own size."""
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    path = models[spec]
    ref = ReferenceLlama(GGUFReader(path), n_ctx=256)
    emu = ReferenceLlama(GGUFReader(path), n_ctx=256)
    eng = _engine(path)
    rng = np.random.default_rng(0)
    toks = [int(t) for t in rng.integers(0, ref.hp.n_vocab, 44)]
    got_pre = eng.eval_logits(toks[:39], 0)
    assert rel_err(got_pre, ref.forward(toks[:39], 0).numpy()) < 5e-2, spec
    e = rel_err(got_pre, emu.forward(toks[:39], 0, path="prefill").numpy())
    assert e < TIGHT[spec], (spec, "prefill", e)
    for i in range(39, 44):   # several graph-replayed decode steps on the prefilled cache
        ref_dec = ref.forward([toks[i]], i).numpy()
        got_dec = eng.decode_logits(toks[i], i)
        assert rel_err(got_dec, ref_dec) < 5e-2, spec
        e = rel_err(got_dec, emu.forward([toks[i]], i, path="decode").numpy())
        assert e < TIGHT[spec], (spec, "decode", i, e)
    assert np.argmax(got_dec) == np.argmax(ref_dec) or \
        ref_dec[np.argmax(got_dec)] > ref_dec.max() - 0.05 * np.abs(ref_dec).max()


# engine vs the rounding-emulating reference over several layers: the emulation reproduces each
# layer op for op (test_one_layer_paths_match_emulation), but 1e-7 differences of f32 summation
# order flip q8 / bf16 roundings in later layers (measured 2-10e-3 at 3-4 layers); MoE: a
# router near-tie flips an expert on one side only
TIGHT = {s: 1.5e-2 for s in SPECS}
TIGHT["tiny-mixtral-q4_k_m"] = 3e-2

ONE_LAYER = ["tiny-llama3-1l", "tiny-mixed-1l", "tiny-q8-1l", "tiny-mixtral-1l"]


@pytest.mark.parametrize("spec", ONE_LAYER)
def test_one_layer_paths_match_emulation(tmp_path, spec):
    """One layer (every quant type across the specs, MoE included): the prefill GEMM path, the
    graph-replayed GEMV decode path and the batched MFMA path each reproduce the reference that
    emulates their rounding - most evaluations to the last bit (< 1e-4), the rest within a
    couple of q8 rounding flips (one flipped head-input element moves the logits ~1e-3: the
    engine's f32 sums differ from torch's in the 7th digit) - where the exact model is 4-7e-3
    away. A wrong sub-block scale, a swapped gate/up row or a lost residual fails every one."""
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = write_synthetic_gguf(spec, str(tmp_path / f"{spec}.gguf"), seed=6)
    emu = ReferenceLlama(GGUFReader(path), n_ctx=128)
    toks = [int(t) for t in np.random.default_rng(2).integers(3, 500, 30)]
    eng = _engine(path, n_ctx=128)
    errs = [("prefill", rel_err(eng.eval_logits(toks[:20], 0), emu.forward(toks[:20], 0, path="prefill").numpy()))]
    for i in range(20, 25):
        errs.append((f"decode{i}", rel_err(eng.decode_logits(toks[i], i),
                                           emu.forward([toks[i]], i, path="decode").numpy())))
    # batched rows (two slots at different lengths); B = 2 takes the batched projections
    beng = load_hip().Engine(path, n_ctx=128, n_batch=64, device=0, use_graph=True, n_slots=3)
    ppath = "prefill16" if beng.prefill_t16 else "prefill"
    if spec in ("tiny-llama3-1l", "tiny-mixtral-1l"):   # batching on: prompts run on the tile16 copies
        assert beng.prefill_t16, spec
    errs.append((ppath, rel_err(beng.eval_logits(toks[:20], 0),
                                ReferenceLlama(GGUFReader(path), n_ctx=128).forward(toks[:20], 0, path=ppath).numpy())))
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    seqs = {0: toks[:9], 2: toks[:14]}
    for s in seqs:
        seqs[s] = seqs[s] + [beng.slot_begin(s, seqs[s], 0, greedy)]
    for step in range(2):
        out = beng.batch_step([0, 2])
        lg = beng.batch_logits(2)
        for b, s in enumerate((0, 2)):
            n = len(seqs[s])
            em = ReferenceLlama(GGUFReader(path), n_ctx=128)
            em.forward(seqs[s][:n - 1 - step], 0, path=ppath)
            for i in range(n - 1 - step, n - 1):
                em.forward([seqs[s][i]], i, path="batch")
            errs.append((f"batch{step}.{s}", rel_err(lg[b], em.forward([seqs[s][n - 1]], n - 1, path="batch").numpy())))
            seqs[s].append(out[b])
    exact_bits = sum(e < 1e-4 for _, e in errs)
    assert exact_bits >= 0.6 * len(errs) and all(e < 3e-3 for _, e in errs), errs


def test_deep_model_no_drift(tmp_path):
    """32 layers (d 1024, Q4_K_M mix incl. the bumped Q6_K V / down layers): prefill and
    decode logits stay within the rounding-flip noise of the emulating reference through the
    whole depth (no accumulating drift)."""
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    path = write_synthetic_gguf("tiny-llama3-deep32", str(tmp_path / "deep.gguf"), seed=2)
    emu = ReferenceLlama(GGUFReader(path), n_ctx=128)
    eng = _engine(path, n_ctx=128)
    toks = [int(t) for t in np.random.default_rng(9).integers(3, 500, 24)]
    e = rel_err(eng.eval_logits(toks[:20], 0), emu.forward(toks[:20], 0, path="prefill").numpy())
    assert e < 1.5e-2, ("prefill", e)
    for i in range(20, 24):
        e = rel_err(eng.decode_logits(toks[i], i), emu.forward([toks[i]], i, path="decode").numpy())
        assert e < 1.5e-2, ("decode", i, e)


@pytest.mark.parametrize("spec", ["tiny-llama3-q4_k_m", "tiny-mixtral-q4_k_m", "tiny-q8-oddff"])
def test_attention_weight_touch_is_transparent(models, spec, monkeypatch):
    """The decode attention's weight-touch plane (LFK_ATTN_TOUCH: this layer's Wo) only reads
    weights: decode logits match the untouched launch up to the fp32 order of the split-K atomics."""
    path = models[spec]
    toks = [int(t) for t in np.random.default_rng(3).integers(0, 1000, 24)]
    logits = []
    for mode in ("0", "1"):
        monkeypatch.setenv("LFK_ATTN_TOUCH", mode)
        eng = _engine(path)
        eng.eval_logits(toks[:20], 0)
        logits.append([eng.decode_logits(toks[i], i) for i in range(20, 23)])
        assert eng.healthy
    for other in logits[1:]:
        for a, b in zip(logits[0], other):
            assert rel_err(a, b) < 1e-2, (spec, rel_err(a, b))


def test_moe_routing_inside_gate_up_matches_router_launch(tmp_path, monkeypatch):
    """Single-row MoE decode at Mixtral's width (d = 4096, 8 experts, top-2): every block of the
    gate/up GEMV routes the token itself (LFK_MOE_ROUTE_FUSE=1, the default) instead of a router
    launch before it. The routing is summed in the router kernel's order (bit-identical picks),
    so the logits match the two-launch form up to the split-K atomics' fp32 order (which flips
    q8 roundings of the next activations: ~1e-2, as test_attention_weight_touch_is_transparent),
    eager and graph, and stay within the fp32 decode emulation's tolerance."""
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    path = write_synthetic_gguf("tiny-mixtral-d4k", str(tmp_path / "mx4k.gguf"), seed=6)
    toks = [int(t) for t in np.random.default_rng(8).integers(3, 1000, 28)]
    out = {}
    for mode, graph in (("0", False), ("1", False), ("1", True)):
        monkeypatch.setenv("LFK_MOE_ROUTE_FUSE", mode)
        eng = _engine(path, graph=graph)
        eng.eval_logits(toks[:20], 0)
        out[(mode, graph)] = [eng.decode_logits(toks[i], i) for i in range(20, 26)]
        assert eng.healthy
        del eng
    for key in (("1", False), ("1", True)):
        for a, b in zip(out[("0", False)], out[key]):
            assert rel_err(b, a) < 1e-2, (key, rel_err(b, a))
    emu = ReferenceLlama(GGUFReader(path), n_ctx=256)
    emu.forward(toks[:20], 0, path="prefill")
    for j, i in enumerate(range(20, 26)):
        e = rel_err(out[("1", True)][j], emu.forward([toks[i]], i, path="decode").numpy())
        assert e < 1.5e-2, ("decode", i, e)


def test_moe_grouped_prefill_chunked(models):
    """Grouped expert prefill (device-side routing, per-expert row counts) is independent of
    how the prompt is chunked: n_batch 16 (3 chunks, partial last) == n_batch 128 (one chunk)."""
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = models["tiny-mixtral-q4_k_m"]
    prompt = [int(t) for t in np.random.default_rng(5).integers(3, 1000, 40)]
    outs = []
    for nb in (16, 128):
        eng = load_hip().Engine(path, n_ctx=256, n_batch=nb, device=0, use_graph=True)
        r = eng.generate(prompt, 0, 12, {"temperature": 0.0}, [], None, None)
        outs.append(r["tokens"])
    assert outs[0] == outs[1]


def test_graph_equals_eager(models):
    path = models["tiny-llama3-q4_k_m"]
    outs = []
    for graph in (True, False):
        eng = _engine(path, graph=graph)
        r = eng.generate([1, 2, 3, 4, 5], 0, 48, {"temperature": 1.0, "top_k": 40, "top_p": 0.95, "seed": 7},
                         [], None, None)
        outs.append(r["tokens"])
    assert outs[0] == outs[1]
    assert len(outs[0]) == 48


def test_prefix_reuse_and_chunked_prefill(models):
    path = models["tiny-llama3-mixed"]
    eng = _engine(path)
    prompt = list(range(10, 210))  # > n_batch (128): two prefill chunks
    sp = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    a = eng.generate(prompt, 0, 16, sp, [], None, None)
    b = eng.generate(prompt, 150, 16, sp, [], None, None)  # reuse 150 cached positions
    assert a["tokens"] == b["tokens"]
    assert b["n_prefilled"] == 50


def test_facade_chat_on_gpu(models):
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    llm = Llama(models["tiny-llama3-q4_k_m"], n_gpu_layers=-1, n_ctx=256, seed=1)
    assert llm.backend_name == "hip"
    out = llm.create_chat_completion([{"role": "user", "content": "hello there"},
                                      {"role": "system", "content": "be brief"}],
                                     temperature=1.2, top_p=0.9, frequency_penalty=0.7, presence_penalty=0.8)
    assert out["usage"]["completion_tokens"] >= 1
    assert out["usage"]["prompt_tokens"] + out["usage"]["completion_tokens"] <= 256
    assert out["timings"]["decode_s"] >= 0


def test_cancel_poll_stops_generation(models):
    eng = _engine(models["tiny-llama3-q4_k_m"], n_ctx=512)
    calls = {"n": 0}

    def poll():
        calls["n"] += 1
        return calls["n"] >= 3
    r = eng.generate([1, 2, 3], 0, 400, {"temperature": 1.0, "seed": 1}, [], poll, None)
    assert r["finish"] == "cancelled" and len(r["tokens"]) < 400


@pytest.mark.parametrize("spec", ["tiny-llama3-q4_k_m", "tiny-mixtral-q4_k_m"])
def test_hybrid_partial_offload_matches_full_gpu(models, spec):
    """n_gpu_layers < n_layer: CPU layers [0, k) + GPU layers [k, n) == all-GPU logits."""
    from llama_fastapi_k8s_gpu_amd.runtime import load_cpu, load_hip
    path = models[spec]
    full = _engine(path, graph=False)
    rng = np.random.default_rng(5)
    toks = [int(t) for t in rng.integers(3, 300, 24)]
    want = full.eval_logits(toks, 0)
    want_dec = full.decode_logits(9, 24)
    cpu = load_cpu().CpuEngine(path, n_ctx=256, n_threads=4, n_batch=16, layer_end=1, load_head=False)
    gpu = load_hip().Engine(path, n_ctx=256, n_batch=128, device=0, use_graph=False, layer_begin=1)
    got = gpu.eval_hidden(cpu.eval_hidden(toks, 0), 0)
    got_dec = gpu.eval_hidden(cpu.eval_hidden([9], 24), 24)
    assert rel_err(got, want) < 3e-2
    assert rel_err(got_dec, want_dec) < 3e-2


def test_hybrid_backend_facade(models):
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    llm = Llama(models["tiny-llama3-q4_k_m"], n_gpu_layers=2, n_ctx=128, seed=4)
    assert llm.backend_name == "hybrid"
    out = llm.create_chat_completion([{"role": "user", "content": "hi"}], max_tokens=8, temperature=0.0)
    assert 1 <= out["usage"]["completion_tokens"] <= 8
    assert llm.health()["cpu_layers"] == 2


def test_facade_sampler_options_on_gpu(models):
    """The HIP backend's routing: logit bias / tail-free / typical stay on the device
    sampler; mirostat, log-probabilities and unlimited top-k take the host loop over
    the engine's logits; a stop string ends the device loop through its poll."""
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    llm = Llama(models["tiny-llama3-q4_k_m"], n_gpu_layers=-1, n_ctx=256, seed=3, verbose=False)
    assert llm.backend_name == "hip"
    forced = 77
    out = llm.create_completion("hello", max_tokens=5, temperature=0.0, logit_bias={forced: 1e4})
    assert llm.tokenize(out["choices"][0]["text"].encode(), add_bos=False) == [forced] * 5 or \
        out["choices"][0]["text"] == llm.detokenize([forced] * 5).decode("utf-8", errors="replace")
    for kw in ({"tfs_z": 0.9}, {"typical_p": 0.8}, {"mirostat_mode": 2}, {"top_k": 0, "top_p": 0.9},
               {"logprobs": 2}):
        r = llm.create_completion("a b c", max_tokens=6, temperature=0.9, seed=4, **kw)
        assert 1 <= r["usage"]["completion_tokens"] <= 6, kw
        if "logprobs" in kw:
            lp = r["choices"][0]["logprobs"]
            assert all(x <= 1e-6 for x in lp["token_logprobs"])
    # grammar-constrained sampling runs on the host loop over the device logits
    g = llm.create_completion("answer:", max_tokens=6, temperature=0.8, seed=2, grammar='root ::= "yes" | "no"')
    assert g["choices"][0]["text"] in ("yes", "no") and g["choices"][0]["finish_reason"] == "stop"
    # host loop (greedy + logprobs) and device loop (greedy) produce the same tokens
    a = llm.create_completion("the quick", max_tokens=8, temperature=0.0, logprobs=1)
    b = llm.create_completion("the quick", max_tokens=8, temperature=0.0)
    assert a["choices"][0]["text"] == b["choices"][0]["text"]
    full = llm.create_completion("the quick", max_tokens=32, temperature=0.0)
    text = full["choices"][0]["text"]
    if len(text) >= 12:
        stop = text[len(text) // 2: len(text) // 2 + 3]
        r = llm.create_completion("the quick", max_tokens=32, temperature=0.0, stop=[stop])
        assert r["choices"][0]["text"] == text[:text.find(stop)]
        assert r["choices"][0]["finish_reason"] == "stop"
        assert r["usage"]["completion_tokens"] < full["usage"]["completion_tokens"]


@pytest.mark.parametrize("on_device", [False, True])
def test_save_load_state_and_device_cache(models, on_device):
    """KV snapshots through host memory and through HBM (strided hipMemcpy2D both ways):
    a restored state continues exactly like the original; the device prompt cache
    restores the longest-prefix conversation."""
    from llama_fastapi_k8s_gpu_amd.engine import LlamaDeviceCache
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    llm = Llama(models["tiny-llama3-q4_k_m"], n_gpu_layers=-1, n_ctx=256, seed=1, verbose=False)
    llm.create_completion("one two three four five", max_tokens=6, temperature=0.0)
    st = llm.save_state(on_device=on_device)
    assert hasattr(st.llama_state, "data_ptr") == on_device
    a = llm.create_completion(list(st.input_ids) + [5], max_tokens=6, temperature=0.0)
    llm.create_completion("something else entirely", max_tokens=6, temperature=0.0)
    llm.load_state(st)
    b = llm.create_completion(list(st.input_ids) + [5], max_tokens=6, temperature=0.0)
    assert a["choices"][0]["text"] == b["choices"][0]["text"] and b["timings"]["n_prefilled"] == 1
    if on_device:
        llm.set_cache(LlamaDeviceCache())
        conv = "alpha beta gamma delta epsilon"
        r1 = llm.create_completion(conv, max_tokens=3, temperature=0.0)
        llm.create_completion("unrelated", max_tokens=3, temperature=0.0)
        cont = conv + r1["choices"][0]["text"] + " zeta"
        r2 = llm.create_completion(cont, max_tokens=2, temperature=0.0)
        assert r2["timings"]["n_prefilled"] < len(llm.tokenize(cont.encode())) - 4
