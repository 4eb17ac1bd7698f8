"""Cycle accounting of one persistent decode step (LFK_PDECODE_ACCT=1): shader-clock totals
per CU kept in registers, so the measurement itself adds no memory traffic."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["item_code", "item_wait", "csync", "sweeps", "items", "attention", "merge", "whole",
         "ld_blocked", "ld_landing", "ld_issue", "unit_loads", "unit_dots", "unit_reduce"]


def main():
    import numpy as np

    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    os.environ["LFK_PDECODE"] = "1"
    os.environ["LFK_PDECODE_ACCT"] = "1"
    model = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b-q4_k_m"
    eng = load_hip().Engine(cached_synthetic_gguf(model), n_ctx=1024, n_batch=512, device=0, use_graph=True)
    toks = [int(t) for t in np.random.default_rng(0).integers(0, 1000, 260)]
    eng.eval_logits(toks[:256], 0)
    for i in range(3):
        eng.decode_logits(toks[256 + i], 256 + i)
    ac = np.asarray(eng.pdecode_acct(), dtype=np.float64).reshape(-1, 16)
    res = {"model": model}
    for i, n in enumerate(NAMES):
        col = ac[:, i]
        res[n] = [round(float(np.median(col)), 1), round(float(col.max()), 1)]
    items = np.median(ac[:, 4])
    res["cycles_per_item_code"] = round(float(np.median(ac[:, 0]) / items), 1)
    res["cycles_per_item_wait"] = round(float(np.median(ac[:, 1]) / items), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
