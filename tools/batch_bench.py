"""Continuous-batching step timing (no HTTP): fill B KV slots with prompts, then time
``batch_step`` over B rows for B in a sweep, next to the single-slot graph decode.
Prints one JSON line; ``--eager-only`` limits the run to the batched path (for rocprofv3)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--n-ctx", type=int, default=1024)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=300)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--batches", default="1,2,4,6,8")
    args = ap.parse_args()
    import numpy as np
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = cached_synthetic_gguf(args.model)
    hip = load_hip()
    eng = hip.Engine(path, n_ctx=args.n_ctx, n_batch=512, device=0, use_graph=True, n_slots=args.slots)
    rng = np.random.default_rng(0)
    sp = {"temperature": 1.2, "top_p": 0.9, "frequency_penalty": 0.7, "presence_penalty": 0.8, "seed": 1}
    res = {"model": args.model, "slots": args.slots, "prompt": args.prompt, "steps": args.steps}
    t0 = time.perf_counter()
    for s in range(args.slots):
        prompt = [int(t) for t in rng.integers(0, eng.hparams["n_vocab"], args.prompt)]
        eng.slot_begin(s, prompt, 0, sp)
    res["slot_begin_ms"] = round((time.perf_counter() - t0) * 1e3 / args.slots, 2)
    # joint admission: the same prompts prefilled together (packed chunks of n_batch rows)
    prompts = [[int(t) for t in rng.integers(0, eng.hparams["n_vocab"], args.prompt)] for _ in range(args.slots)]
    t0 = time.perf_counter()
    eng.slots_begin(list(range(args.slots)), prompts, [0] * args.slots, [sp] * args.slots)
    res["slots_begin_ms_per_prompt"] = round((time.perf_counter() - t0) * 1e3 / args.slots, 2)
    for B in [int(b) for b in args.batches.split(",")]:
        if B > eng.max_batch:
            continue
        slots = list(range(B))
        eng.batch_step(slots)  # warm
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.batch_step(slots)
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        res[f"B{B}_ms_per_step"] = round(ms, 3)
        res[f"B{B}_tok_s"] = round(B / ms * 1e3, 1)
        if getattr(eng, "can_pipeline", False):
            # the scheduler's mode: step k + 1 queued before step k's tokens are collected
            t0 = time.perf_counter()   # exactly args.steps steps launched and collected in here
            eng.batch_launch(slots)
            for _ in range(args.steps - 1):
                eng.batch_launch(slots)
                eng.batch_collect()
            eng.batch_collect()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            res[f"B{B}_pipelined_ms_per_step"] = round(ms, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
