"""The tensor-parallel control channel (csrc/runtime/tp_channel.h) across processes:
rank 0 publishes commands, followers receive every one of them in order (the mailbox
is never overwritten before every follower copied it), a follower that attaches late
sees only what comes after, and a follower notices a leader that died."""
import multiprocessing as mp
import os
import time

import pytest


def _name(tag):
    return f"lfk_test_{tag}_{os.getpid()}_{os.urandom(3).hex()}"


def _follower(name, rank, n, q):
    from llama_fastapi_k8s_gpu_amd.runtime import load_cpu
    cpu = load_cpu()
    c = cpu.TPChannel.attach(name, rank)
    q.put(("ready", rank))
    got = []
    while True:
        m = c.receive(5000)
        if m is None:
            q.put(("timeout", rank, got))
            return
        if m == b"STOP":
            break
        got.append(m)
        if len(got) % 7 == 0:
            time.sleep(0.01)   # a slow follower: the leader must wait for its copy
    q.put(("done", rank, got))


def test_channel_order_and_backpressure():
    from llama_fastapi_k8s_gpu_amd.runtime import load_cpu
    cpu = load_cpu()
    world, n = 3, 200
    name = _name("order")
    lead = cpu.TPChannel.create(name, world, 4096)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_follower, args=(name, r, n, q)) for r in range(1, world)]
    for p in procs:
        p.start()
    for _ in procs:
        assert q.get(timeout=60)[0] == "ready"
    msgs = [bytes([i % 251]) * (1 + (i * 37) % 3000) for i in range(n)]
    for m in msgs:
        lead.publish(m)
    lead.publish(b"STOP")
    res = [q.get(timeout=60) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for kind, rank, got in res:
        assert kind == "done", (kind, rank)
        assert got == msgs, rank


def _orphan(name, q):
    from llama_fastapi_k8s_gpu_amd.runtime import load_cpu
    c = load_cpu().TPChannel.attach(name, 1)
    q.put("attached")
    deadline = time.time() + 30
    while time.time() < deadline:
        if c.receive(200) is None and not c.leader_alive():
            q.put("leader gone")
            return
    q.put("still waiting")


def _leader_then_exit(name, q):
    from llama_fastapi_k8s_gpu_amd.runtime import load_cpu
    c = load_cpu().TPChannel.create(name, 2, 64)
    q.put("created")
    time.sleep(1.0)
    os._exit(0)   # dies without publishing STOP (and without unlinking)


def test_follower_detects_dead_leader():
    name = _name("dead")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    lp = ctx.Process(target=_leader_then_exit, args=(name, q))
    lp.start()
    assert q.get(timeout=60) == "created"
    fp = ctx.Process(target=_orphan, args=(name, q))
    fp.start()
    assert q.get(timeout=60) == "attached"
    assert q.get(timeout=60) == "leader gone"
    lp.join(timeout=10)
    fp.join(timeout=10)
    # the orphaned follower removed the dead leader's segment when its channel closed
    assert not os.path.exists("/dev/shm/" + name)


def _attach_then_exit(name, q):
    from llama_fastapi_k8s_gpu_amd.runtime import load_cpu
    c = load_cpu().TPChannel.attach(name, 1)   # noqa: F841 (kept open until the process dies)
    q.put("attached")
    q.close()
    q.join_thread()   # the message is out before the process dies
    os._exit(0)   # a follower that crashes without consuming anything


def test_leader_detects_dead_follower():
    """A follower that died fails the leader's next publish within a fraction of a second
    (its pid is probed while the leader waits for the mailbox), not after the 600 s timeout."""
    from llama_fastapi_k8s_gpu_amd.runtime import load_cpu
    cpu = load_cpu()
    name = _name("deadf")
    lead = cpu.TPChannel.create(name, 2, 64)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    fp = ctx.Process(target=_attach_then_exit, args=(name, q))
    fp.start()
    assert q.get(timeout=60) == "attached"
    fp.join(timeout=30)
    lead.publish(b"one")           # the mailbox was empty: nothing to wait for
    t0 = time.time()
    with pytest.raises(Exception, match="exited"):
        lead.publish(b"two")       # waits for the dead follower's copy of "one"
    assert time.time() - t0 < 10


def test_channel_rejects_bad_use():
    from llama_fastapi_k8s_gpu_amd.runtime import load_cpu
    cpu = load_cpu()
    with pytest.raises(Exception):
        cpu.TPChannel.attach(_name("missing"), 1)
    name = _name("cap")
    lead = cpu.TPChannel.create(name, 2, 16)
    with pytest.raises(Exception):
        lead.publish(b"x" * 17)             # larger than the mailbox
    with pytest.raises(Exception):
        cpu.TPChannel.create(name, 2, 16)   # the name is taken
    assert lead.world == 2
