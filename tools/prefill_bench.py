"""Single-prompt admission prefill as the bench's continuous batch runs it (engine with the
production n_slots = 7: tile16 copies, tile16 prefill GEMMs): ``slot_begin`` of one T-token prompt
(prefill + first token) repeated on fresh slots, and ``slots_begin`` of 6 prompts jointly.
Prints one JSON line; run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel table.

    python tools/prefill_bench.py [--T 387] [--reps 8]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--T", type=int, default=387)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--joint", type=int, default=6)
    args = ap.parse_args()
    import numpy as np
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    path = cached_synthetic_gguf(args.model)
    eng = load_hip().Engine(path, n_ctx=1024, n_batch=512, device=0, use_graph=True, n_slots=7)
    rng = np.random.default_rng(0)
    sp = {"temperature": 1.2, "top_p": 0.9, "frequency_penalty": 0.7, "presence_penalty": 0.8, "seed": 1}
    V = eng.hparams["n_vocab"]
    prompts = [[int(t) for t in rng.integers(0, V, args.T)] for _ in range(args.reps + 1)]
    eng.slot_begin(1, prompts[-1], 0, sp)  # warm (first-use allocations)
    ts = []
    for i in range(args.reps):
        t0 = time.perf_counter()
        eng.slot_begin(1 + i % 6, prompts[i], 0, sp)
        ts.append((time.perf_counter() - t0) * 1e3)
    res = {"model": args.model, "T": args.T, "prefill_t16": bool(getattr(eng, "prefill_t16", False)),
           "slot_begin_ms": [round(t, 2) for t in ts], "slot_begin_ms_med": round(float(np.median(ts)), 2)}
    if args.joint > 1:
        jp = [[int(t) for t in rng.integers(0, V, args.T)] for _ in range(args.joint)]
        eng.slots_begin(list(range(1, 1 + args.joint)), jp, [0] * args.joint, [sp] * args.joint)
        jp = [[int(t) for t in rng.integers(0, V, args.T)] for _ in range(args.joint)]
        t0 = time.perf_counter()
        eng.slots_begin(list(range(1, 1 + args.joint)), jp, [0] * args.joint, [sp] * args.joint)
        res["joint_admission_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        res["joint_prompts"] = args.joint
    print(json.dumps(res))


if __name__ == "__main__":
    main()
