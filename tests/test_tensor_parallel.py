"""Tensor-parallel shard plan validated without GPUs.

The C++ CPU backend runs the same shard plan as the GPU engine
(csrc/runtime/shard.h: column-split Q/K/V and gate/up, row-split Wo and down,
vocab-split lm_head) with its collectives over a gloo process group, one
process per rank exactly like the RCCL deployment. TP=2 logits must match the
TP=1 logits up to float summation order (every cut is on a q8 block boundary,
so no extra quantisation error is introduced beyond rounding flips).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
from llama_fastapi_k8s_gpu_amd.runtime import load_cpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, path, tokens, out_dir, split):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from llama_fastapi_k8s_gpu_amd.parallel.comm import host_collectives
        cpu = load_cpu()
        ts = list(split or [])
        eng = cpu.CpuEngine(path, n_ctx=64, n_threads=2, n_batch=8, tp_rank=rank, tp_size=world, tensor_split=ts)
        eng.set_comm(*host_collectives())
        a = eng.eval_logits(tokens, 0)
        b = eng.eval_logits([5], len(tokens))      # one decode step on top of the prefill
        sp = {"top_k": 40, "top_p": 0.9, "min_p": 0.05, "temperature": 1.2, "repeat_penalty": 1.1,
              "frequency_penalty": 0.7, "presence_penalty": 0.8, "last_n": 64, "seed": 9}
        eng2 = cpu.CpuEngine(path, n_ctx=64, n_threads=2, n_batch=8, tp_rank=rank, tp_size=world, tensor_split=ts)
        eng2.set_comm(*host_collectives())
        g = eng2.generate(tokens, 0, 6, sp, [])
        np.save(os.path.join(out_dir, f"r{rank}_a.npy"), a)
        np.save(os.path.join(out_dir, f"r{rank}_b.npy"), b)
        np.save(os.path.join(out_dir, f"r{rank}_g.npy"), np.array(g["tokens"], np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model,world,split", [
    ("tiny-llama3-tp", 2, None), ("tiny-mixtral-tp", 2, None),
    ("tiny-llama3-tp4", 2, [3, 1]),     # llama.cpp tensor_split proportions: 3 of 4 kv heads / FFN superblocks
    ("tiny-llama3-tp4", 2, [1, 2]),
    ("tiny-llama3-tp4", 3, None),       # degree not dividing the heads: apportioned 2/1/1
])
def test_tp_matches_tp1(tmp_path, model, world, split):
    path = write_synthetic_gguf(model, str(tmp_path / f"{model}.gguf"))
    rng = np.random.default_rng(0)
    tokens = [int(t) for t in rng.integers(3, 400, 12)]
    cpu = load_cpu()
    ref = cpu.CpuEngine(path, n_ctx=64, n_threads=2, n_batch=8)
    want_a = ref.eval_logits(tokens, 0)
    want_b = ref.eval_logits([5], len(tokens))
    mp.start_processes(_rank_main, args=(world, _free_port(), path, tokens, str(tmp_path), split), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        a = np.load(tmp_path / f"r{r}_a.npy")
        b = np.load(tmp_path / f"r{r}_b.npy")
        assert a.shape == want_a.shape
        # partial sums meet in a different order (and a rounding flip in a later
        # per-32 q8 activation block can follow): compare at the q8 noise level
        for got, want in ((a, want_a), (b, want_b)):
            assert np.linalg.norm(got - want) / np.linalg.norm(want) < 5e-3
            assert int(np.argmax(got)) == int(np.argmax(want))
    # every rank samples the same tokens (identical gathered logits + shared seed)
    for r in range(1, world):
        assert np.array_equal(np.load(tmp_path / "r0_g.npy"), np.load(tmp_path / f"r{r}_g.npy"))


def test_shard_plan_rejects_bad_degree(tmp_path):
    path = write_synthetic_gguf("tiny-llama3-tp", str(tmp_path / "m.gguf"))
    cpu = load_cpu()
    with pytest.raises(RuntimeError, match="exceeds the kv-head count"):
        cpu.CpuEngine(path, n_ctx=32, tp_rank=0, tp_size=5)
    with pytest.raises(RuntimeError, match="superblock-aligned"):   # 4 kv heads of 128 q columns: pairs
        cpu.CpuEngine(path, n_ctx=32, tp_rank=0, tp_size=3)
    with pytest.raises(RuntimeError, match="entries for"):
        cpu.CpuEngine(path, n_ctx=32, tp_rank=0, tp_size=2, tensor_split=[1.0, 1.0, 1.0])
    with pytest.raises(RuntimeError, match="set_comm"):
        cpu.CpuEngine(path, n_ctx=32, tp_rank=0, tp_size=2).eval_logits([1, 2], 0)


def test_tensor_split_validation():
    from llama_fastapi_k8s_gpu_amd.parallel.comm import check_tensor_split
    assert check_tensor_split(None, 2) == []
    assert check_tensor_split([0.7, 0.3], 2) == [0.7, 0.3]
    assert check_tensor_split([0.5, 0.5, 0, 0], 2) == [0.5, 0.5]   # trailing unused GPUs
    with pytest.raises(ValueError, match="positive weight"):
        check_tensor_split([1, 1, 1], 2)
    with pytest.raises(ValueError, match="positive weight"):
        check_tensor_split([1, 0, 1], 3)


def _serve_rank(rank, world, port, path, out_dir):
    """rank 0: FastAPI app with the TP leader; rank 1: follower loop (CPU backend, gloo)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from llama_fastapi_k8s_gpu_amd.config import Settings
    from llama_fastapi_k8s_gpu_amd.engine.factory import build_engine
    from llama_fastapi_k8s_gpu_amd.parallel.tp_serve import TPLeader, follower_loop, init_tp
    import torch.distributed as dist
    s = Settings()
    s.model_path_override = path
    s.n_gpu_layers = 0
    s.n_ctx = 256
    r, w, ctrl = init_tp(s)
    assert (r, w) == (rank, world) and s.split_mode == "row" and s.seed is not None
    llm = build_engine(s)
    assert llm.health()["tp"] == 2
    if rank == 0:
        from fastapi.testclient import TestClient
        from llama_fastapi_k8s_gpu_amd.server.app import create_app
        leader = TPLeader(llm, ctrl)
        with TestClient(create_app(s, engine=leader)) as c:
            body = {"bot_profile": {"name": "Ann.f", "appearance": "a, b, c, d"}, "user_profile": {"name": "u"},
                    "context": [{"turn": "user", "message": "hello there"}]}
            codes = [c.post("/response", json=body).status_code for _ in range(2)]
        leader.close()
        with open(os.path.join(out_dir, "codes.txt"), "w") as f:
            f.write(",".join(map(str, codes)))
    else:
        follower_loop(llm, ctrl)
        open(os.path.join(out_dir, "follower_done"), "w").close()
    dist.destroy_process_group()


def test_tp_serving_leader_follower(tmp_path):
    path = write_synthetic_gguf("tiny-llama3-tp", str(tmp_path / "m.gguf"))
    mp.start_processes(_serve_rank, args=(2, _free_port(), path, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    assert (tmp_path / "codes.txt").read_text() == "200,200"
    assert (tmp_path / "follower_done").exists()
