"""Per-XCD block timeline of ONE layer of the batched decode step, in the step's own context
(the engine passes wall_clock64 stamp buffers to that layer's kernels: LFK_STEP_CLK=<layer>).

wall_clock64 is not aligned across XCDs, so every number is taken within one XCD (blocks
stamp their XCC id): per kernel and XCD the first block start and the last block end; the
gap between consecutive kernels on the same XCD is the kernel boundary as the XCD sees it.

    LFK_STEP_CLK=5 python tools/step_blocks.py [--rows 6] [--prompt 700] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["qkv", "attn", "wo", "gate_up", "down"]
# stamp meaning per kernel kind: bmm [0 entry, 1 weights issued, 2 x staged, 3 first tile, 4 exit, 5 tiles,
# 6 xcc]; attention [0 entry, 1 loads+pos, 2 V staged, 3 scores, 4 partials met, 5 partial stored,
# 6 counter, 8 merge start, 9 merge end, 15 xcc]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--rows", type=int, default=6)
    ap.add_argument("--prompt", type=int, default=700)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    if "LFK_STEP_CLK" not in os.environ:
        os.environ["LFK_STEP_CLK"] = "5"
    import numpy as np
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import cached_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    eng = hip.Engine(cached_synthetic_gguf(args.model), n_ctx=1024, n_batch=512, device=0, use_graph=True,
                     n_slots=max(8, args.rows))
    rng = np.random.default_rng(0)
    sp = {"temperature": 1.2, "top_p": 0.9, "seed": 1}
    slots = list(range(args.rows))
    prompts = [[int(t) for t in rng.integers(0, eng.hparams["n_vocab"], args.prompt)] for _ in slots]
    eng.slots_begin(slots, prompts, [0] * len(slots), [sp] * len(slots))
    for _ in range(args.steps):
        eng.batch_step(slots)
    eng.step_clk_zero()
    eng.batch_step(slots)
    clk = eng.step_clk()
    res = {"rows": args.rows, "prompt": args.prompt, "layer": int(os.environ["LFK_STEP_CLK"])}
    us = lambda t: float(t) / 100.0  # noqa: E731 (100 MHz)
    per = {}
    for k, name in enumerate(NAMES):
        c = clk[k] if name == "attn" else clk[k].reshape(-1, 8)   # bmm stamps: 8 per block
        live = c[:, 0] > 0
        xcc_col = 15 if name == "attn" else 6
        c = c[live]
        if len(c) == 0:
            continue
        xcc = (c[:, xcc_col] & 0xF).astype(int)
        ends = np.where(c[:, :15] > 0, c[:, :15], 0).max(axis=1) if name == "attn" else c[:, 4].copy()
        ends = np.where(ends > 0, ends, c[:, :5].max(axis=1))
        life = ends - c[:, 0]
        d = {"blocks": int(len(c)), "life_us_p50_p90_max": [round(us(np.percentile(life, 50)), 2),
                                                             round(us(np.percentile(life, 90)), 2),
                                                             round(us(life.max()), 2)]}
        for j, lab in ((1, "s1"), (2, "s2"), (3, "s3")):
            v = c[:, j] - c[:, 0]
            v = v[c[:, j] > 0]
            if len(v):
                d[lab + "_us_p50_p90"] = [round(us(np.percentile(v, 50)), 2), round(us(np.percentile(v, 90)), 2)]
        if name == "attn":
            m = c[:, 8] > 0
            if m.any():
                d["merge_start_us_p50"] = round(us(np.percentile(c[m, 8] - c[m, 0], 50)), 2)
                d["merge_dur_us_p50"] = round(us(np.percentile(c[m, 9] - c[m, 8], 50)), 2)
        spans = {}
        for x in sorted(set(xcc.tolist())):
            sel = xcc == x
            spans[x] = (int(c[sel, 0].min()), int(ends[sel].max()), int(np.percentile(c[sel, 0], 90)))
        d["span_us_per_xcd"] = [round(us(e - s), 2) for s, e, _ in spans.values()]
        d["start_spread_p90_us_per_xcd"] = [round(us(p - s), 2) for s, _, p in spans.values()]
        per[name] = (d, spans)
        res[name] = d
    # kernel boundaries per XCD: next kernel's first start - this kernel's last end
    order = [n for n in NAMES if n in per]
    for a, b in zip(order, order[1:]):
        gaps = [us(per[b][1][x][0] - per[a][1][x][1]) for x in per[a][1] if x in per[b][1]]
        res[f"gap_{a}_{b}_us"] = [round(g, 2) for g in gaps]
    # layer time per XCD: first qkv start -> last down end
    if "qkv" in per and "down" in per:
        res["layer_us_per_xcd"] = [round(us(per["down"][1][x][1] - per["qkv"][1][x][0]), 2)
                                   for x in per["qkv"][1] if x in per["down"][1]]
    print(json.dumps(res, indent=1), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
