"""Engine logits vs the rounding-emulating reference (models/llama.py ReferenceLlama path=...)
per path and step, for a few tiny models: the residual after emulation, and the exact-model
error it replaces. Prints one JSON line per model."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    from gpu_helpers import rel_err
    from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    from llama_fastapi_k8s_gpu_amd.models.llama import ReferenceLlama
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    specs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["tiny-llama3-q4_k_m", "tiny-llama3-mixed",
                                                               "tiny-tinyllama-q8_0", "tiny-llama3-wide"]
    d = tempfile.mkdtemp()
    for spec in specs:
        path = write_synthetic_gguf(spec, os.path.join(d, spec + ".gguf"), seed=3)
        eng = load_hip().Engine(path, n_ctx=256, n_batch=128, device=0, use_graph=True)
        ref = ReferenceLlama(GGUFReader(path), n_ctx=256)
        emu = ReferenceLlama(GGUFReader(path), n_ctx=256)
        toks = [int(t) for t in np.random.default_rng(0).integers(0, ref.hp.n_vocab, 48)]
        r = {"spec": spec}
        # one token at position 0: the GEMVs and a one-key attention only
        g0 = eng.decode_logits(toks[0], 0)
        r["decode_pos0"] = [round(rel_err(g0, emu.forward([toks[0]], 0, path="decode").numpy()), 6),
                            round(rel_err(g0, ref.forward([toks[0]], 0).numpy()), 6)]
        g = eng.eval_logits(toks[:39], 0)
        r["prefill"] = [round(rel_err(g, emu.forward(toks[:39], 0, path="prefill").numpy()), 5),
                        round(rel_err(g, ref.forward(toks[:39], 0).numpy()), 5)]
        dec = []
        for i in range(39, 48):
            g = eng.decode_logits(toks[i], i)
            dec.append([round(rel_err(g, emu.forward([toks[i]], i, path="decode").numpy()), 5),
                        round(rel_err(g, ref.forward([toks[i]], i).numpy()), 5)])
        r["decode"] = dec
        # batched rows: two slots, one batched step each (B = 2: the bmm projections)
        beng = load_hip().Engine(path, n_ctx=256, n_batch=128, device=0, use_graph=True, n_slots=3)
        greedy = {"temperature": 0.0, "top_k": 1, "repeat_penalty": 1.0}
        seqs = {0: toks[:9], 2: toks[:14]}
        for s_ in seqs:
            seqs[s_] = seqs[s_] + [beng.slot_begin(s_, seqs[s_], 0, greedy)]
        beng.batch_step([0, 2])
        lg = beng.batch_logits(2)
        bt = []
        for b, s_ in enumerate((0, 2)):
            n = len(seqs[s_])
            em = ReferenceLlama(GGUFReader(path), n_ctx=256)
            em.forward(seqs[s_][:n - 1], 0, path="prefill")
            bt.append(round(rel_err(lg[b], em.forward([seqs[s_][n - 1]], n - 1, path="batch").numpy()), 6))
        r["batch"] = bt
        if ref.hp.n_expert:  # router-weight variant: f32 instead of bf16 in the prefill GEMM
            em = ReferenceLlama(GGUFReader(path), n_ctx=256)
            em._bf16_router = False
            orig = em._bf16
            for L in em.layers:
                L["ffn_gate_inp_f32"] = L["ffn_gate_inp"]
            g = eng.eval_logits(toks[:39], 0)
            em._bf16 = lambda x: x if any(x is L["ffn_gate_inp"] for L in em.layers) else orig(x)
            r["prefill_router_f32"] = round(rel_err(g, em.forward(toks[:39], 0, path="prefill").numpy()), 6)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
