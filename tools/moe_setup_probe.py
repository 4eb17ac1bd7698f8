"""Single-row decode logits of an MoE model with the batched-MoE setup on and off (the setup
only builds tile16 copies: the single-row path must not change)."""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(path, out):
    import numpy as np
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    eng = load_hip().Engine(path, n_ctx=256, n_batch=64, device=0, use_graph=True, n_slots=4)
    toks = [int(t) for t in np.random.default_rng(11).integers(3, 400, 48)]
    res = [eng.eval_logits(toks[:39], 0)] + [eng.decode_logits(toks[39 + i], 39 + i) for i in range(6)]
    np.save(out, np.stack(res))


if __name__ == "__main__":
    if len(sys.argv) == 3:
        run(sys.argv[1], sys.argv[2])
        sys.exit(0)
    import numpy as np
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    d = tempfile.mkdtemp()
    for spec in sys.argv[1].split(","):
        path = write_synthetic_gguf(spec, os.path.join(d, spec + ".gguf"), seed=4)
        outs = []
        for moe in ("0", "1"):
            o = os.path.join(d, f"{spec}_{moe}.npy")
            subprocess.run([sys.executable, __file__, path, o], check=True, env=dict(os.environ, LFK_BATCH_MOE=moe))
            outs.append(np.load(o))
        diff = np.abs(outs[0] - outs[1]).max(axis=1) / np.abs(outs[0]).max(axis=1)
        print(spec, [round(float(v), 6) for v in diff], "nan:", bool(np.isnan(outs[1]).any()), flush=True)
