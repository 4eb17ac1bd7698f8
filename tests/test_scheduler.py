"""Continuous-batching scheduler (csrc/runtime/scheduler.cpp) on the CPU, over a
deterministic multi-slot stand-in engine (``_cpu.FakeSlotEngine``): every request's
tokens must equal a sequential run of the same request, whatever else shares the
batch; prefix reuse, queueing past the slot count, cancellation, the context end and
device errors are covered. The MI355X engine runs the same scheduler object
(tests/test_batch_gpu.py checks the batched numerics)."""
import threading
import time

import pytest

from llama_fastapi_k8s_gpu_amd.runtime import load_cpu

VOCAB = 997


def sequential(prompt, max_new, n_ctx, stop_ids=()):
    """The token stream one request gets on its own (the fake's next-token rule)."""
    nt = load_cpu().FakeSlotEngine.next_token
    seq = list(prompt)
    out = [nt(seq, VOCAB)]
    while True:
        t = out[-1]
        if t in stop_ids or len(out) >= max_new or len(prompt) + len(out) - 1 >= n_ctx:
            return out
        seq.append(t)
        out.append(nt(seq, VOCAB))


def run(sched, rid, timeout=20.0):
    toks, t0 = [], time.time()
    while time.time() - t0 < timeout:
        r = sched.wait(rid, len(toks), 50)
        toks += r["tokens"]
        if r["done"]:
            sched.release(rid)
            return toks, r
    raise AssertionError("request did not finish")


PIPELINE = {"on": False}


@pytest.fixture(autouse=True, params=[False, True], ids=["sync", "pipelined"])
def _pipeline(request):
    """Every scheduler test runs twice: synchronous batch_step, and the pipelined
    batch_launch / batch_collect loop (the next step queued before this one's tokens are
    handled - the MI355X engine's mode)."""
    PIPELINE["on"] = request.param
    yield


def make(n_slots=5, max_batch=4, n_ctx=64, step_us=200):
    cpu = load_cpu()
    eng = cpu.FakeSlotEngine(n_slots, max_batch, n_ctx, VOCAB, step_us)
    eng.set_pipeline(PIPELINE["on"])
    return eng, cpu.BatchScheduler(eng)


def test_batched_rows_match_sequential_runs():
    eng, sched = make()
    reqs = [([1, 2, 3, 4 + i], 10 + 3 * i) for i in range(4)]
    ids = [sched.submit(p, m, {}, []) for p, m in reqs]
    for rid, (p, m) in zip(ids, reqs):
        toks, r = run(sched, rid)
        assert toks == sequential(p, m, 64), rid
        assert r["finish"] == "length" and r["n_prefilled"] == len(p)
    assert eng.max_rows == 4        # the four requests decoded as one batch
    st = sched.stats()
    assert st["admitted"] == 4 and st["active"] == 0 and st["pending"] == 0
    sched.shutdown()


def test_more_requests_than_slots_queue_and_finish():
    eng, sched = make(n_slots=3, max_batch=8)   # two scheduler slots (slot 0 is reserved)
    reqs = [([5, i, i + 1], 6 + i) for i in range(7)]
    ids = [sched.submit(p, m, {}, []) for p, m in reqs]
    for rid, (p, m) in zip(ids, reqs):
        toks, _ = run(sched, rid)
        assert toks == sequential(p, m, 64)
    assert eng.max_rows <= 2
    sched.shutdown()


def test_stop_ids_and_context_end():
    eng, sched = make(n_ctx=32)
    p = [9, 8, 7]
    ref = sequential(p, 1000, 32)
    stop = ref[5]
    toks, r = run(sched, sched.submit(p, 1000, {}, [stop]))
    assert toks == ref[:ref.index(stop) + 1] and r["finish"] == "stop"
    long_prompt = list(range(1, 30))       # 29 of 32 positions: 4 tokens fit (the last is never fed)
    toks, r = run(sched, sched.submit(long_prompt, 1000, {}, []))
    assert len(toks) == 32 - 29 + 1 and r["finish"] == "length"
    assert toks == sequential(long_prompt, 1000, 32)
    sched.shutdown()


def test_prefix_reuse_across_requests():
    eng, sched = make(n_slots=3, max_batch=2)
    p1 = list(range(10, 40))
    t1, _ = run(sched, sched.submit(p1, 8, {}, []))
    before = eng.prefilled
    # the follow-up turn: the whole previous conversation plus new text
    p2 = p1 + t1[:-1] + [t1[-1], 77, 78]
    t2, r2 = run(sched, sched.submit(p2, 5, {}, []))
    assert t2 == sequential(p2, 5, 64)
    resident = len(p1) + len(t1) - 1       # the last sampled token was never fed
    assert r2["n_prefilled"] == len(p2) - resident
    assert eng.prefilled - before == len(p2) - resident
    assert sched.stats()["reused_tokens"] == resident
    sched.shutdown()


def test_cancel_frees_the_slot_and_others_continue():
    eng, sched = make(n_slots=3, max_batch=2, n_ctx=4096, step_us=2000)
    a = sched.submit([1, 2, 3], 100000, {}, [])
    b = sched.submit([4, 5, 6], 40, {}, [])
    time.sleep(0.05)
    sched.cancel(a)
    ta, ra = run(sched, a)
    assert ra["finish"] == "cancelled" and 0 < len(ta) < 100000
    c = sched.submit([7, 8], 5, {}, [])     # takes a's freed slot while b still runs
    tc, _ = run(sched, c)
    tb, rb = run(sched, b)
    assert tb == sequential([4, 5, 6], 40, 4096) and rb["finish"] == "length"
    assert tc == sequential([7, 8], 5, 4096)
    sched.shutdown()


def test_engine_error_ends_the_batch_rows_and_scheduler_survives():
    eng, sched = make(n_slots=3, max_batch=2)
    eng.fail_at(3)
    toks, r = run(sched, sched.submit([1, 2], 50, {}, []))
    assert r["finish"] == "error" and "injected" in r["error"]
    toks, r = run(sched, sched.submit([3, 4], 5, {}, []))   # later requests still run
    assert r["finish"] == "length" and toks == sequential([3, 4], 5, 64)
    sched.shutdown()


def test_concurrent_submitters_and_shutdown():
    eng, sched = make(n_slots=9, max_batch=8, n_ctx=256, step_us=100)
    results, errs = {}, []

    def client(i):
        try:
            p = [i + 1, 2 * i + 3, 11]
            toks, _ = run(sched, sched.submit(p, 20 + i, {}, []))
            results[i] = toks == sequential(p, 20 + i, 256)
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(e)
    th = [threading.Thread(target=client, args=(i,)) for i in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(30)
    assert not errs and len(results) == 16 and all(results.values())
    assert eng.max_rows > 1
    pending = sched.submit([1, 2, 3], 10 ** 6, {}, [])
    sched.shutdown()
    r = sched.wait(pending, 0, 1000)
    assert r["done"] and r["finish"] == "cancelled"
    with pytest.raises(RuntimeError):
        sched.submit([1], 1, {}, [])


def test_requests_queued_together_are_admitted_together():
    """Requests that queue while a step runs are admitted in one slots_begin call (one packed
    prefill on the MI355X engine); their tokens still equal their sequential runs."""
    eng, sched = make(n_slots=5, max_batch=4, n_ctx=256, step_us=3000)
    first = sched.submit([1, 2, 3], 50, {}, [])
    time.sleep(0.02)                       # the scheduler is inside a 3 ms step now
    reqs = [([7, i, 9, 10 + i], 12) for i in range(3)]
    ids = [sched.submit(p, m, {}, []) for p, m in reqs]
    for rid, (p, m) in zip(ids, reqs):
        toks, r = run(sched, rid)
        assert toks == sequential(p, m, 256) and r["n_prefilled"] == len(p)
    run(sched, first)
    st = sched.stats()
    assert st["joint_admissions"] >= 1 and st["admitted"] == 4
    sched.shutdown()


def test_long_prompt_admitted_in_parts_between_decode_steps():
    """Chunked admission: a prompt longer than the engine's prefill chunk that arrives while
    rows decode is prefilled part by part between their steps (the rows keep stepping while it
    loads), and its tokens - like the decoding rows' - equal the sequential runs; a prompt
    arriving on an idle engine is admitted whole; a reused prefix is not prefilled again."""
    eng, sched = make(n_slots=4, max_batch=3, n_ctx=256, step_us=1000)
    eng.set_prefill_chunk(16)
    first_p = [3, 1, 4, 1, 5]
    first = sched.submit(first_p, 60, {}, [])
    got = sched.wait(first, 0, 5000)       # `first` is decoding now (its first token is out)
    assert got["tokens"] and not got["done"]
    steps0 = eng.steps
    long_p = list(range(100, 170))         # 70 tokens: 5 parts of 16
    rid = sched.submit(long_p, 8, {}, [])
    toks, r = run(sched, rid)
    assert toks == sequential(long_p, 8, 256) and r["n_prefilled"] == len(long_p)
    assert eng.parts >= 5
    assert eng.steps - steps0 >= 4         # the decoding row stepped while the prompt loaded
    ftoks, _ = run(sched, first)
    assert ftoks == sequential(first_p, 60, 256)
    st = sched.stats()
    assert st["chunked_admissions"] == 1 and st["admitted"] == 2
    # the follow-up turn on the now idle engine reuses the long prompt's resident prefix
    p2 = long_p + toks[:-1] + [toks[-1], 9, 9]
    t2, r2 = run(sched, sched.submit(p2, 4, {}, []))
    assert t2 == sequential(p2, 4, 256)
    assert r2["n_prefilled"] == len(p2) - (len(long_p) + len(toks) - 1)
    sched.shutdown()


def test_cancel_while_prefilling_in_parts():
    eng, sched = make(n_slots=4, max_batch=3, n_ctx=512, step_us=2000)
    eng.set_prefill_chunk(8)
    first = sched.submit([1, 2], 200, {}, [])
    assert sched.wait(first, 0, 5000)["tokens"]           # decoding
    rid = sched.submit(list(range(10, 300)), 5, {}, [])   # 37 parts
    time.sleep(0.01)
    sched.cancel(rid)
    r = sched.wait(rid, 0, 5000)
    while not r["done"]:
        r = sched.wait(rid, 0, 5000)
    assert r["finish"] == "cancelled"
    # the slot is free again: another long request is admitted and completes
    p = list(range(400, 440))
    toks, _ = run(sched, sched.submit(p, 6, {}, []))
    assert toks == sequential(p, 6, 512)
    sched.cancel(first)
    sched.shutdown()


def test_cancelled_part_admission_does_not_leave_a_stale_prefix():
    """A chunked admission overwrites its slot's KV from the reused prefix on. Cancelled
    mid-prefill, the slot must not still advertise the previous occupant's history: a later
    prompt extending that history may reuse only the prefix both requests shared (the fake
    engine raises 'reused prefix differs' otherwise)."""
    eng, sched = make(n_slots=3, max_batch=2, n_ctx=512, step_us=2000)
    eng.set_prefill_chunk(8)
    p = list(range(50, 90))
    ta, _ = run(sched, sched.submit(p, 3, {}, []))         # idle engine: admitted whole, slot s
    first = sched.submit([1, 2], 400, {}, [])              # decodes in the other slot
    assert sched.wait(first, 0, 5000)["tokens"]
    q = p[:10] + list(range(600, 890))                     # shares 10 tokens with p: slot s, keep 10
    rid = sched.submit(q, 5, {}, [])
    time.sleep(0.01)
    sched.cancel(rid)
    r = sched.wait(rid, 0, 5000)
    while not r["done"]:
        r = sched.wait(rid, 0, 5000)
    assert r["finish"] == "cancelled"
    sched.release(rid)
    p2 = p + ta[:-1] + [ta[-1], 7, 7]                      # the follow-up turn of the first request
    t2, r2 = run(sched, sched.submit(p2, 4, {}, []))
    assert r2["finish"] == "length", r2.get("error")
    assert t2 == sequential(p2, 4, 512)
    sched.cancel(first)
    sched.shutdown()
