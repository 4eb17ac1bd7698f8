"""Eager persistent decode steps of a BASELINE model for rocprofv3 (kernel trace or
PMC counters): the graph path is invisible to rocprofv3's kernel trace.

    rocprofv3 --kernel-trace --stats -d gpurun_out/pdprof -- python3 tools/pdecode_prof.py
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--off", action="store_true", help="launch-per-op decode instead")
    args = ap.parse_args()
    import numpy as np

    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    os.environ["LFK_PDECODE"] = "0" if args.off else "1"
    path = cached_synthetic_gguf(args.model)
    eng = load_hip().Engine(path, n_ctx=1024, n_batch=512, device=0, use_graph=False)
    print("pdecode:", eng.pdecode, file=sys.stderr, flush=True)
    toks = [int(t) for t in np.random.default_rng(0).integers(0, 1000, args.prompt + args.steps)]
    eng.eval_logits(toks[:args.prompt], 0)
    for i in range(args.steps):
        eng.decode_logits(toks[args.prompt + i], args.prompt + i)
    print("healthy:", eng.healthy, eng.last_error, file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
