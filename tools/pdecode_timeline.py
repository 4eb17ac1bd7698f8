"""Stage timeline of one persistent decode step (LFK_PDECODE_TIMELINE=1).

Stamps per CU and layer (wall clock, 100 MHz): 0 layer start, 1 x gathered, 2 QKV
consumed, 3 o gathered (attention + merge + hand-off), 4 Wo consumed, 5 x gathered
(ffn), 6 gate/up consumed, 7 h gathered, 8 down consumed; loader: 10 first item
issued, 11 last item issued. Prints median / p90 / max over CUs of every stage span (us)
for the middle layers, and the whole step."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["gather_x", "qkv", "attn_gather_o", "wo", "gather_x2", "gate_up", "gather_h", "down"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--prompt", type=int, default=256)
    args = ap.parse_args()
    import numpy as np

    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    os.environ["LFK_PDECODE"] = "1"
    os.environ["LFK_PDECODE_TIMELINE"] = "1"
    path = cached_synthetic_gguf(args.model)
    eng = load_hip().Engine(path, n_ctx=1024, n_batch=512, device=0, use_graph=True)
    assert eng.pdecode == "on", eng.pdecode
    hp = eng.hparams
    toks = [int(t) for t in np.random.default_rng(0).integers(0, 1000, args.prompt + 4)]
    eng.eval_logits(toks[:args.prompt], 0)
    for i in range(3):
        eng.decode_logits(toks[args.prompt + i], args.prompt + i)
    raw = np.asarray(eng.pdecode_timeline(), dtype=np.int64)
    ncu = raw.size // (hp["n_layer"] * 12 + 48 * 8)
    tl = raw[:ncu * hp["n_layer"] * 12].reshape(ncu, hp["n_layer"], 12).astype(np.float64) / 100.0  # us
    ti = raw[ncu * hp["n_layer"] * 12:].reshape(ncu, 48, 8).astype(np.float64) / 100.0
    t0 = tl[:, 0, 0].min()
    res = {"model": args.model, "ncu": ncu, "healthy": bool(eng.healthy), "error": eng.last_error,
           "step_us": round(float(tl[:, -1, 8].max() - t0), 1)}
    mid = slice(2, hp["n_layer"] - 2)
    for i, name in enumerate(NAMES):
        span = tl[:, mid, i + 1] - tl[:, mid, i]
        res[name] = [round(float(np.median(span)), 2), round(float(np.percentile(span, 90)), 2),
                     round(float(span.max()), 2)]
    layer = tl[:, 3:, 0].min(axis=0) - tl[:, 2:-1, 0].min(axis=0)
    res["layer_us_median"] = round(float(np.median(layer)), 2)
    # loader: how far ahead of the consumers does it issue a layer's first item
    res["loader_lead_us"] = round(float(np.median(tl[:, mid, 0] - tl[:, mid, 10])), 2)
    res["loader_layer_issue_span_us"] = round(float(np.median(tl[:, mid, 11] - tl[:, mid, 10])), 2)
    print(json.dumps(res), flush=True)
    # items of layer 2, relative to the layer start of each CU: loader issue, consumer wait
    # start, item available, released (median over CUs)
    base = tl[:, 2, 0][:, None]
    nit = int((ti[0, :, 0] > 0).sum())
    rows = []
    for k in range(nit):
        rows.append([k] + [round(float(np.median(ti[:, k, c] - base[:, 0])), 2) for c in (0, 2, 3, 4)])
    print(json.dumps({"items_layer2_median_us[k, issue, wait, avail, released]": rows}), flush=True)


if __name__ == "__main__":
    main()
