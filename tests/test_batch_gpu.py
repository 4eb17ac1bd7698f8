"""Continuous batching on the MI355X engine (KV slots, ``slot_begin`` / ``batch_step``):
every row of a batched decode step (MFMA GEMMs over the rows, per-row RoPE + KV append
into its own slot, batched split-L attention, lm_head GEMM, batched GPU sampler) must
match the fp32 reference model on that row's own sequence, with the slots at different
lengths; the sampler's greedy pick is the argmax of the row's logits."""
import numpy as np
import pytest

from gpu_helpers import rel_err

pytestmark = pytest.mark.gpu

SPECS = ["tiny-llama3-q4_k_m", "tiny-tinyllama-q8_0", "tiny-mixtral-q4_k_m"]


@pytest.fixture(scope="module")
def models(tmp_path_factory):
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    d = tmp_path_factory.mktemp("batch_models")
    return {s: write_synthetic_gguf(s, str(d / f"{s}.gguf")) for s in SPECS}


@pytest.mark.parametrize("spec", SPECS)
def test_batch_step_rows_match_reference(models, spec):
    from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = models[spec]
    eng = load_hip().Engine(path, n_ctx=256, n_batch=64, device=0, use_graph=False, n_slots=4)
    assert eng.n_slots == 4 and eng.max_batch == 4
    ref = ReferenceLlama(GGUFReader(path), n_ctx=256)
    emu = ReferenceLlama(GGUFReader(path), n_ctx=256)
    rng = np.random.default_rng(3)
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    slots = [3, 0, 1]                      # not in order, slot 2 unused
    seqs, plen, paths = {}, {}, {}
    for s, n in zip(slots, (5, 40, 17)):
        prompt = [int(t) for t in rng.integers(3, 300, n)]
        first = eng.slot_begin(s, prompt, 0, greedy)
        seqs[s] = prompt + [first]
        plen[s] = n
        paths[s] = []

    def emulated(s):
        """The slot's history as the engine computed it: the prompt on the prefill path, each
        fed token on the path of the step that fed it (batched rows; one row = the GEMV decode)."""
        out = emu.forward(seqs[s][:plen[s]], 0, path="prefill16" if eng.prefill_t16 else "prefill")
        for i, p in enumerate(paths[s]):
            out = emu.forward([seqs[s][plen[s] + i]], plen[s] + i, path=p)
        return out.numpy()
    for step in range(3):
        toks = eng.batch_step(slots)
        logits = eng.batch_logits(len(slots))
        for b, s in enumerate(slots):
            paths[s].append("batch")
            want = ref.forward(seqs[s], 0).numpy()
            assert rel_err(logits[b], want) < 5e-2, (spec, step, s, rel_err(logits[b], want))
            e = rel_err(logits[b], emulated(s))
            assert e < TIGHT[spec], (spec, step, s, e)
            assert toks[b] == int(np.argmax(logits[b]))
            seqs[s].append(toks[b])
    # a sub-batch of the slots continues where each slot stands (one row: the GEMV decode graph)
    toks = eng.batch_step([1])
    paths[1].append("decode")
    want = ref.forward(seqs[1], 0).numpy()
    assert rel_err(eng.batch_logits(1)[0], want) < 5e-2
    assert rel_err(eng.batch_logits(1)[0], emulated(1)) < TIGHT[spec]
    assert eng.healthy, eng.last_error


# the rounding-flip noise of several layers (see test_engine_gpu.TIGHT); one layer is checked
# op for op in test_engine_gpu.test_one_layer_paths_match_emulation
TIGHT = {"tiny-llama3-q4_k_m": 1.5e-2, "tiny-tinyllama-q8_0": 1.5e-2, "tiny-mixtral-q4_k_m": 3e-2}


def test_batch_step_d4096_fused_paths(tmp_path):
    """d = 4096 (the 8B width, 4 layers): the batched step runs the folded RMSNorm (Q|K|V and
    gate/up stage fp32 rows), the SwiGLU epilogue and, on the bumped layers (Q6_K Wv), the
    Q|K + V two-type launch - rows against the fp32 reference."""
    from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = write_synthetic_gguf("pd-llama-g4", str(tmp_path / "g4.gguf"))
    eng = load_hip().Engine(path, n_ctx=128, n_batch=64, device=0, use_graph=True, n_slots=4)
    ref = ReferenceLlama(GGUFReader(path), n_ctx=128)
    emu = ReferenceLlama(GGUFReader(path), n_ctx=128)
    rng = np.random.default_rng(5)
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    seqs, plen = {}, {}
    for s, n in zip((2, 0, 3), (6, 11, 9)):
        prompt = [int(t) for t in rng.integers(3, 300, n)]
        seqs[s] = prompt + [eng.slot_begin(s, prompt, 0, greedy)]
        plen[s] = n
    for rows in ([2, 0, 3], [0, 3]):
        toks = eng.batch_step(rows)
        logits = eng.batch_logits(len(rows))
        for b, s in enumerate(rows):
            want = ref.forward(seqs[s], 0).numpy()
            assert rel_err(logits[b], want) < 5e-2, (s, rel_err(logits[b], want))
            out = emu.forward(seqs[s][:plen[s]], 0, path="prefill16" if eng.prefill_t16 else "prefill")
            for i in range(plen[s], len(seqs[s])):
                out = emu.forward([seqs[s][i]], i, path="batch")
            e = rel_err(logits[b], out.numpy())
            assert e < 1.5e-2, (s, e)
            assert toks[b] == int(np.argmax(logits[b]))
            seqs[s].append(toks[b])
    assert eng.healthy, eng.last_error


@pytest.mark.parametrize("joint_rows", ["default", "0"])
@pytest.mark.parametrize("spec", ["tiny-llama3-q4_k_m", "tiny-mixtral-q4_k_m"])
def test_joint_admission_matches_sequential(models, spec, joint_rows, monkeypatch):
    """slots_begin packs several prompts into shared prefill chunks (per-row KV slot and
    position, every prompt piece of a chunk in one attention launch; one prompt reuses its slot's
    resident prefix): first tokens and the rows of the following batched steps equal slot-by-slot
    admission. Default: the whole admission in one pass (Engine::kJointRows); LFK_JOINT_ROWS=0:
    chunks of n_batch = 32 rows, so pieces cross chunk boundaries."""
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    if joint_rows != "default":
        monkeypatch.setenv("LFK_JOINT_ROWS", joint_rows)
    kw = dict(n_ctx=256, n_batch=32, device=0, use_graph=False, n_slots=4)
    joint, seq = hip.Engine(models[spec], **kw), hip.Engine(models[spec], **kw)
    monkeypatch.delenv("LFK_JOINT_ROWS", raising=False)
    rng = np.random.default_rng(12)
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    base = [int(t) for t in rng.integers(3, 300, 21)]
    for e in (joint, seq):                 # slot 1 holds `base`: the second round reuses it
        e.slot_begin(1, base, 0, greedy)
    prompts = [[int(t) for t in rng.integers(3, 300, n)] for n in (45, 7)] + [base + [11, 12, 13]]
    slots, keep = [3, 0, 1], [0, 0, len(base)]
    a = joint.slots_begin(slots, prompts, keep, [greedy] * 3)
    b = [seq.slot_begin(s, p, k, greedy) for s, p, k in zip(slots, prompts, keep)]
    assert a == b
    for _ in range(3):
        ta, tb = joint.batch_step(slots), seq.batch_step(slots)
        la, lb = joint.batch_logits(3), seq.batch_logits(3)
        for r in range(3):
            assert rel_err(la[r], lb[r]) < 1e-3, (r, rel_err(la[r], lb[r]))
        assert ta == tb
    assert joint.healthy, joint.last_error


def test_batch_sampling_params_are_per_slot(models):
    """Each slot samples with its own parameters, penalty ring and seed."""
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    eng = load_hip().Engine(models["tiny-llama3-q4_k_m"], n_ctx=256, n_batch=64, device=0, use_graph=False,
                            n_slots=3)
    prompt = [5, 6, 7, 8, 9]
    forced = 123
    eng.slot_begin(0, prompt, 0, {"temperature": 0.0, "top_k": 1, "logit_bias": {forced: 1e4}})
    eng.slot_begin(1, prompt, 0, {"temperature": 1.0, "top_k": 40, "top_p": 0.9, "seed": 7})
    eng.slot_begin(2, prompt, 0, {"temperature": 1.0, "top_k": 40, "top_p": 0.9, "seed": 7})
    outs = {0: [], 1: [], 2: []}
    for _ in range(6):
        t = eng.batch_step([0, 1, 2])
        for b in range(3):
            outs[b].append(t[b])
    assert outs[0] == [forced] * 6
    assert outs[1] == outs[2]              # same prompt, params and seed: same draws
    assert all(0 <= t < 16256 for t in outs[1])


def test_single_slot_engine_rejects_batching(models):
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    eng = load_hip().Engine(models["tiny-llama3-q4_k_m"], n_ctx=128, n_batch=32, device=0, use_graph=False)
    with pytest.raises(RuntimeError):
        eng.batch_step([0])


def test_pipelined_steps_equal_synchronous(models):
    """batch_launch / batch_collect (step k + 1 queued before step k's tokens are read, the
    scheduler's mode) produce exactly the tokens of synchronous batch_step calls - the steps
    feed from device-resident tokens - including a one-row step (the single-row graph) and a
    row set change."""
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = models["tiny-llama3-q4_k_m"]
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    rng = np.random.default_rng(8)
    prompts = {s: [int(t) for t in rng.integers(3, 300, n)] for s, n in ((1, 7), (2, 19), (3, 12))}
    plan = [[1, 2, 3]] * 4 + [[2]] * 3 + [[1, 3]] * 3

    def run(pipelined):
        eng = load_hip().Engine(path, n_ctx=256, n_batch=64, device=0, use_graph=True, n_slots=4)
        assert eng.can_pipeline
        first = {s: eng.slot_begin(s, p, 0, greedy) for s, p in prompts.items()}
        out = []
        if not pipelined:
            for rows in plan:
                out.append(list(eng.batch_step(rows)))
        else:
            i = 0
            while i < len(plan):
                eng.batch_launch(plan[i])
                if i + 1 < len(plan) and plan[i + 1] == plan[i]:
                    eng.batch_launch(plan[i + 1])
                    out.append(list(eng.batch_collect()))
                    out.append(list(eng.batch_collect()))
                    i += 2
                else:
                    out.append(list(eng.batch_collect()))
                    i += 1
        assert eng.healthy, eng.last_error
        return first, out
    assert run(False) == run(True)


@pytest.mark.parametrize("joint", [False, True])
def test_slot_begin_while_steps_in_flight(models, joint):
    """The scheduler admits a request (slot_begin / slots_begin) while a pipelined step is still
    queued - into a slot whose row that very step is computing (its request just ended): the
    admission's state upload and prefill are ordered behind the in-flight step on the engine
    stream, so the new request's first token and every later step equal a run that collected
    the step first."""
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = models["tiny-llama3-q4_k_m"]
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    rng = np.random.default_rng(12)
    prompts = {s: [int(t) for t in rng.integers(3, 300, n)] for s, n in ((1, 9), (2, 14), (3, 11))}
    newp = [int(t) for t in rng.integers(3, 300, 17)]

    def run(overlap):
        eng = load_hip().Engine(path, n_ctx=256, n_batch=64, device=0, use_graph=True, n_slots=4)
        for s, p in prompts.items():
            eng.slot_begin(s, p, 0, greedy)
        out = []
        eng.batch_launch([1, 2, 3])
        eng.batch_launch([1, 2, 3])
        out.append(list(eng.batch_collect()))

        def admit():
            return eng.slots_begin([3], [newp], [0], [greedy])[0] if joint else eng.slot_begin(3, newp, 0, greedy)
        if overlap:
            first = admit()                              # step 2 still queued
            out.append(list(eng.batch_collect())[:2])    # slot 3's token of that step is dropped
        else:
            out.append(list(eng.batch_collect())[:2])
            first = admit()
        for _ in range(4):
            out.append(list(eng.batch_step([1, 2, 3])))
        assert eng.healthy, eng.last_error
        return first, out
    assert run(True) == run(False)


def test_chunked_admission_equals_whole(models):
    """slot_begin_part (the scheduler's chunked admission: prompt parts between other rows'
    decode steps) gives the same first token and the same following batched rows as slot_begin,
    with a batch step of another slot between every two parts and a reused prefix."""
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = models["tiny-llama3-q4_k_m"]
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    rng = np.random.default_rng(21)
    other = [int(t) for t in rng.integers(3, 300, 10)]
    base = [int(t) for t in rng.integers(3, 300, 12)]
    long_p = base + [int(t) for t in rng.integers(3, 300, 75)]

    def run(chunked):
        eng = load_hip().Engine(path, n_ctx=256, n_batch=32, device=0, use_graph=True, n_slots=4)
        assert eng.prefill_part_tokens > 0
        eng.slot_begin(1, other, 0, greedy)
        eng.slot_begin(2, base, 0, greedy)              # slot 2 holds `base`: reused below
        out = []
        if chunked:
            done, first = len(base), -1
            while first < 0:
                first = eng.slot_begin_part(2, long_p, len(base), done, 20, greedy)
                done = min(len(long_p), done + 20)
                out.append(list(eng.batch_step([1])))   # the other row decodes in between
        else:
            first = eng.slot_begin(2, long_p, len(base), greedy)
            for _ in range(4):                          # (20-token parts of 75: 4 parts)
                out.append(list(eng.batch_step([1])))
        out += [list(eng.batch_step([1, 2])) for _ in range(3)]
        assert eng.healthy, eng.last_error
        return first, out
    assert run(True) == run(False)


def test_batch_step_six_rows_d8192(tmp_path):
    """Six rows at d = 8192: the split-K Q|K|V beside the FFN path that does not stage a whole row
    (its projections' inputs prepared by bprep), which must re-zero the split-K rows itself -
    every row of three consecutive steps against the fp32 reference on its own sequence."""
    from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = write_synthetic_gguf("tiny-llama3-d8k", str(tmp_path / "d8k.gguf"))
    eng = load_hip().Engine(path, n_ctx=128, n_batch=64, device=0, use_graph=True, n_slots=7)
    ref = ReferenceLlama(GGUFReader(path), n_ctx=128)
    rng = np.random.default_rng(9)
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    slots = [6, 0, 1, 2, 4, 5]
    seqs = {}
    for s in slots:
        prompt = [int(t) for t in rng.integers(3, 300, 4 + 3 * s)]
        seqs[s] = prompt + [eng.slot_begin(s, prompt, 0, greedy)]
    for step in range(3):
        toks = eng.batch_step(slots)
        logits = eng.batch_logits(len(slots))
        for b, s in enumerate(slots):
            want = ref.forward(seqs[s], 0).numpy()
            assert rel_err(logits[b], want) < 5e-2, (step, s, rel_err(logits[b], want))
            seqs[s].append(toks[b])
    assert eng.healthy, eng.last_error


@pytest.mark.parametrize("n_rows", [9, 12, 16])
def test_batch_step_more_than_eight_rows(models, n_rows):
    """Batches past 8 rows (MAX_BATCH / n_slots > 8): the layers run their 16-row forms and the
    lm_head, whose store-only epilogue takes at most 8 rows per launch, runs in 8-row chunks -
    every row against the fp32 reference, greedy pick = argmax of its logits."""
    from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = models["tiny-llama3-q4_k_m"]
    eng = load_hip().Engine(path, n_ctx=128, n_batch=64, device=0, use_graph=True, n_slots=16)
    assert eng.max_batch == 16
    ref = ReferenceLlama(GGUFReader(path), n_ctx=128)
    rng = np.random.default_rng(30 + n_rows)
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    slots = [int(s) for s in rng.permutation(16)[:n_rows]]
    seqs = {}
    for s in slots:
        prompt = [int(t) for t in rng.integers(3, 300, 3 + s)]
        seqs[s] = prompt + [eng.slot_begin(s, prompt, 0, greedy)]
    for step in range(2):
        toks = eng.batch_step(slots)
        logits = eng.batch_logits(len(slots))
        for b, s in enumerate(slots):
            want = ref.forward(seqs[s], 0).numpy()
            assert rel_err(logits[b], want) < 5e-2, (n_rows, step, s, rel_err(logits[b], want))
            assert toks[b] == int(np.argmax(logits[b]))
            seqs[s].append(toks[b])
    assert eng.healthy, eng.last_error


def test_batched_and_serial_decode_agree_near_n_ctx(models):
    """RoPE from one source on every path: rows decoded batched (deferred RoPE in the batched
    attention, fp32 pos * freq) and the same sequences decoded one at a time (the rope table, built
    from the same fp32 angles) agree at positions near n_ctx = 1024, where a rotation computed two
    ways would drift the most - both against the fp32 reference, and against each other."""
    from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = models["tiny-llama3-q4_k_m"]
    hip = load_hip()
    bat = hip.Engine(path, n_ctx=1024, n_batch=512, device=0, use_graph=True, n_slots=3)
    one = hip.Engine(path, n_ctx=1024, n_batch=512, device=0, use_graph=False)
    ref = ReferenceLlama(GGUFReader(path), n_ctx=1024)
    rng = np.random.default_rng(77)
    greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
    prompts = [[int(t) for t in rng.integers(3, 300, n)] for n in (1010, 990)]
    seqs = []
    for s, p in enumerate(prompts):
        seqs.append(p + [bat.slot_begin(s, p, 0, greedy)])
    for step in range(2):
        toks = bat.batch_step([0, 1])
        lb = bat.batch_logits(2)
        for b in range(2):
            seq = seqs[b]
            # the one-row engine: the same history on its prefill path, then this step's token decoded
            one.eval_logits(seq[:512], 0)
            one.eval_logits(seq[512:-1], 512)
            ls = one.decode_logits(seq[-1], len(seq) - 1)
            want = ref.forward(seq, 0).numpy()
            assert rel_err(lb[b], want) < 5e-2, (step, b, rel_err(lb[b], want))
            assert rel_err(ls, want) < 5e-2, (step, b, rel_err(ls, want))
            assert rel_err(lb[b], ls) < 5e-2, (step, b, rel_err(lb[b], ls))
            assert toks[b] == int(np.argmax(lb[b]))
            seqs[b].append(toks[b])
    assert bat.healthy, bat.last_error
