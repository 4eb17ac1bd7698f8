"""Per-layer, per-stage comparison of the persistent decode step against the fp32
reference model (LFK_PDECODE_DUMP=1 makes the kernel store every layer's
intermediates). Prints one JSON line per layer: relative error of q, k, v,
attention output, x after Wo, SwiGLU output and x after down."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", default="pd-llama-8b2")
    ap.add_argument("--n", type=int, default=20)
    args = ap.parse_args()
    import numpy as np

    from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    os.environ["LFK_PDECODE"] = "1"
    os.environ["LFK_PDECODE_DUMP"] = "1"
    path = cached_synthetic_gguf(args.spec, seed=11)
    eng = load_hip().Engine(path, n_ctx=512, n_batch=128, device=0, use_graph=False)
    print("status", eng.pdecode, file=sys.stderr, flush=True)
    ref = ReferenceLlama(GGUFReader(path), n_ctx=512)
    hp = eng.hparams
    d, hd, nh, nkv, F = hp["n_embd"], hp["head_dim"], hp["n_head"], hp["n_head_kv"], hp["n_ff"]
    nq, nk = nh * hd, nkv * hd
    rng = np.random.default_rng(0)
    toks = [int(t) for t in rng.integers(3, 1000, args.n + 1)]
    for p0 in range(0, args.n, 128):
        eng.eval_logits(toks[p0:min(args.n, p0 + 128)], p0)
    got_logits = np.asarray(eng.decode_logits(toks[args.n], args.n))
    dump = np.asarray(eng.pdecode_dump())
    trace = []
    want_logits = ref.forward(toks[:args.n + 1], 0, trace=trace).numpy()
    stride = 2 * nq + 2 * nk + 2 * d + F
    offs = {"q": (0, nq), "k": (nq, nk), "v": (nq + nk, nk), "o": (nq + 2 * nk, nq), "x_attn": (2 * nq + 2 * nk, d),
            "h": (2 * nq + 2 * nk + d, F), "x_ffn": (2 * nq + 2 * nk + d + F, d)}

    def rel(a, b):
        return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    for li, t in enumerate(trace):
        row = {"layer": li}
        base = li * stride
        for k, (o, n) in offs.items():
            got = dump[base + o: base + o + n]
            want = t[k].numpy().reshape(-1)
            row[k] = round(rel(got, want), 5)
            if row[k] > 0.05:
                bad = np.argsort(-np.abs(got - want))[:4]
                row[k + "_worst"] = [[int(i), float(got[i]), float(want[i])] for i in bad]
        print(json.dumps(row), flush=True)
    print(json.dumps({"logits_rel_err": round(rel(got_logits, want_logits), 5), "healthy": bool(eng.healthy),
                      "error": eng.last_error}), flush=True)


if __name__ == "__main__":
    main()
