"""Write a synthetic GGUF into the benches' model cache (TMPDIR/llama_amd_models, as bench.py and
tools/decode_bench.py read it), printing each tensor as it goes (a 40 GB 70B file takes minutes:
the progress lines keep a GPU session's watchdog fed).
    python tools/gen_model.py llama3-70b-q4_k_m [--seed 0]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    d = os.environ.get("SYNTH_MODEL_DIR") or os.path.join(os.environ.get("TMPDIR", "/tmp"), "llama_amd_models")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"{args.model}-s{args.seed}.gguf")
    if os.path.exists(path):
        print("exists", path, flush=True)
        return
    t0 = time.time()
    write_synthetic_gguf(args.model, path, args.seed, log=lambda n: print(f"{time.time() - t0:7.1f}s {n}", flush=True))
    print(f"wrote {path} ({os.path.getsize(path) / 1e9:.1f} GB) in {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
