"""BASELINE config #1: TinyLlama-1.1B Q8_0 with n_gpu_layers=0 on the C++ CPU
backend, through the FastAPI /response path (synthetic weights and requests)."""
import argparse
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--max-tokens", type=int, default=64)
    args = ap.parse_args()
    from bench import CountingEngine, make_request
    from llama_fastapi_k8s_gpu_amd.config import Settings
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.server.app import create_app
    import httpx
    path = cached_synthetic_gguf("tinyllama-1.1b-q8_0")
    llm = Llama(path, n_gpu_layers=0, n_ctx=1024, seed=1, backend="cpu", n_threads=args.threads or None, verbose=False)
    eng = CountingEngine(llm)
    s = Settings()
    s.timeout_seconds = 600
    s.sampling.max_tokens = args.max_tokens   # bounded: CPU decode of ~700 tokens per request takes minutes
    app = create_app(s, engine=eng)
    lat = []

    async def run():
        async with app.router.lifespan_context(app):
            async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://b", timeout=600) as c:
                t0 = time.perf_counter()
                for i in range(args.steps):
                    t = time.perf_counter()
                    r = await c.post("/response", json=make_request(i))
                    assert r.status_code == 200, r.text
                    lat.append(time.perf_counter() - t)
                return time.perf_counter() - t0
    el = asyncio.run(run())
    toks = sum(eng.completion_tokens)
    dec = sum(eng.decode_s)
    print(json.dumps({"config": "TinyLlama-1.1B Q8_0, n_gpu_layers=0 (C++ CPU backend)", "threads": args.threads or os.cpu_count(),
                      "output_tok_s": round(toks / el, 2), "decode_tok_s": round(toks / dec, 2) if dec else None,
                      "p50_response_ms": round(statistics.median(lat) * 1e3, 1),
                      "avg_prompt_tokens": sum(eng.prompt_tokens) / len(eng.prompt_tokens),
                      "avg_output_tokens": toks / len(eng.completion_tokens), "max_tokens": args.max_tokens}))


if __name__ == "__main__":
    main()
