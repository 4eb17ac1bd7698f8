"""Headline benchmark: output tokens/s + p50 /response latency, Llama-3-8B Q4_K_M
(BASELINE.json metric), measured through the real FastAPI ``/response`` path.

One "step" = one ``POST /response`` request, served exactly as the reference
serves it (reference api.py:118-173): persona system prompt, context
truncation, admission queue, ``create_chat_completion(temperature=1.2,
top_p=0.9, frequency_penalty=0.7, presence_penalty=0.8)`` with no max_tokens -
so each request decodes until EOS or the 1024-token context is full.

Parallelism (one process per GPU, launched by torch.distributed.run for N>1):
  * ``--parallel dp`` (default): every GPU is an independent replica serving its
    own request stream - the reference's deployment model (4 replicas behind one
    Service, reference helm/values.yaml:17). Weak scaling; value = sum over ranks.
  * ``--parallel tp``: one model row-split over all GPUs (RCCL all-reduce over
    xGMI); every rank serves the same requests. Strong scaling; value = rank 0's.

Load: ``--clients C`` concurrent clients (default 6 = the reference pod's admission
capacity, 1 in flight + MAX_QUEUE_SIZE 5, reference api.py:19,113) post the K timed
requests; the engine decodes up to ``--max-batch M`` (default = C) of them as rows of
one continuous batch (csrc/runtime/scheduler.cpp). ``--clients 1 --max-batch 1`` is
the reference's serial one-generation-at-a-time serving (recorded in profiles/).

Weights are random-init of the exact Llama-3-8B Q4_K_M shapes and type mix
(a synthetic GGUF written once per node), prompts are synthetic chat requests.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "output tokens/sec + p50 /response latency, Llama-3-8B Q4_K_M at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # BASELINE.json "published": {} - no reference number exists


class CountingEngine:
    """Delegates to the real engine and records usage per /response."""
    supports_cancel = True

    def __init__(self, llm):
        self.llm = llm
        self.completion_tokens = []
        self.prompt_tokens = []
        self.decode_s = []

    def create_chat_completion(self, **kw):
        out = self.llm.create_chat_completion(**kw)
        self.completion_tokens.append(out["usage"]["completion_tokens"])
        self.prompt_tokens.append(out["usage"]["prompt_tokens"])
        self.decode_s.append(out["timings"]["decode_s"])
        return out

    def health(self):
        return self.llm.health()


def make_request(i: int) -> dict:
    names = ["Mia.f", "Leo", "Ava.f", "Max"]
    ctx = []
    for j in range(6):
        turn = "user" if j % 2 == 0 else "assistant"
        ctx.append({"turn": turn, "message": f"message {i}-{j}: tell me something fun about the number {i * 7 + j} "
                                              "and how you would spend a rainy afternoon in a small seaside town."})
    return {"bot_profile": {"name": names[i % 4], "appearance": "tall, brown hair, green eyes, freckles, smiles"},
            "user_profile": {"name": "bench"}, "context": ctx}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--parallel", choices=["dp", "tp"], default="dp")
    ap.add_argument("--n-ctx", type=int, default=1024)
    ap.add_argument("--clients", type=int, default=6, help="concurrent clients posting /response")
    ap.add_argument("--max-batch", type=int, default=0, help="continuous-batch rows (0 = --clients)")
    ap.add_argument("--model-dir", default=os.environ.get("SYNTH_MODEL_DIR", os.path.join(
        os.environ.get("TMPDIR", "/tmp"), "llama_amd_models")))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal mode: LFK_BENCH_DEVICE=<d> puts every rank on GPU d (a one-GPU box running
    # the N-rank DP flow); RCCL refuses two ranks on one device, so the bench's own barrier
    # and reductions go over gloo then.
    rehearse = os.environ.get("LFK_BENCH_DEVICE")
    if rehearse is not None:
        local = int(rehearse)
        os.environ["LOCAL_RANK"] = str(local)
    torch.cuda.set_device(local)
    if world > 1:
        if rehearse is not None:
            if args.parallel == "tp":
                raise SystemExit("LFK_BENCH_DEVICE rehearses dp only (TP needs one GPU per rank)")
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    red_dev = "cpu" if rehearse is not None else "cuda"

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import SPECS, write_synthetic_gguf
    os.makedirs(args.model_dir, exist_ok=True)
    path = os.path.join(args.model_dir, f"{args.model}-s0.gguf")
    if (rank if rehearse is not None else local) == 0 and not os.path.exists(path):
        t0 = time.time()
        write_synthetic_gguf(args.model, path, seed=0)
        print(f"[bench] wrote synthetic {args.model} in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    barrier()

    from llama_fastapi_k8s_gpu_amd.config import Settings
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    from llama_fastapi_k8s_gpu_amd.server.app import create_app

    t0 = time.time()
    split = "row" if (args.parallel == "tp" and world > 1) else "none"
    max_batch = args.max_batch or args.clients
    if split == "row":
        max_batch = 1   # continuous batching runs on one rank
    llm = Llama(path, n_gpu_layers=-1, n_ctx=args.n_ctx, seed=1234 + (0 if split == "row" else rank),
                split_mode=split, verbose=False, **({"max_batch": max_batch} if max_batch > 1 else {}))
    print(f"[bench] rank {rank}: loaded in {time.time() - t0:.1f}s ({llm.backend_name})", file=sys.stderr,
          flush=True)
    eng = CountingEngine(llm)
    settings = Settings()
    settings.timeout_seconds = 600.0  # measure latency, do not 408 long generations in the bench
    settings.max_batch = max_batch
    settings.max_queue_size = max(settings.max_queue_size, args.clients)
    app = create_app(settings, engine=eng)

    import httpx

    latencies = []

    async def run():
        async with app.router.lifespan_context(app):
            transport = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=transport, base_url="http://bench", timeout=600) as c:
                async def drive(ids, lat):
                    todo = list(ids)

                    async def client():
                        while todo:
                            i = todo.pop(0)
                            t = time.perf_counter()
                            r = await c.post("/response", json=make_request(i))
                            assert r.status_code == 200, r.text
                            if lat is not None:
                                lat.append(time.perf_counter() - t)
                    await asyncio.gather(*[client() for _ in range(max(1, args.clients))])
                await drive(range(1000, 1000 + args.warmup), None)
                barrier()
                n0 = len(eng.completion_tokens)
                t_start = time.perf_counter()
                await drive(range(args.steps), latencies)
                barrier()
                return time.perf_counter() - t_start, n0

    elapsed, n0 = asyncio.run(run())
    llm.close()
    toks = sum(eng.completion_tokens[n0:])
    ptoks = sum(eng.prompt_tokens[n0:])
    if world > 1:
        t = torch.tensor([elapsed, float(toks if (args.parallel == "dp" or rank == 0) else 0)],
                         dtype=torch.float64, device=red_dev)
        tmax = t[0].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, total = float(tmax), float(t[1])
    else:
        total = float(toks)
    value = total / elapsed
    p50 = statistics.median(latencies) * 1e3
    dec = sum(eng.decode_s[n0:])
    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "weak" if args.parallel == "dp" else "strong",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None, "dtype": "q4_k_m weights; f16 (batched MFMA) / int8 (single-row GEMV) / bf16 (prefill MFMA) activations; fp32 accumulate",
            "data": "synthetic (random-init Llama-3-8B Q4_K_M GGUF, synthetic chat requests)",
            "config": {"model": "Llama-3-8B Q4_K_M",
                       "global_batch": (world if args.parallel == "dp" else 1) * min(args.clients, max_batch),
                       "seq_len": args.n_ctx, "parallelism": f"{args.parallel}{world}",
                       "clients_per_gpu": args.clients, "max_batch": max_batch,
                       "p50_response_ms": round(p50, 1),
                       "decode_tokens_per_s_per_request": round(toks / dec, 1) if dec > 0 else None,
                       "avg_prompt_tokens": round(ptoks / max(1, args.steps), 1),
                       "avg_output_tokens": round(toks / max(1, args.steps), 1)},
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
