"""Per-block timeline of one decode GEMV launch (instrumented kernel build):
when blocks start, how long the x prologue takes, when the first item and the
whole block finish. Weights stream from HBM (fresh copy, not cache-resident)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

Q4_K, Q6_K = 12, 14


def main():
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    s = torch.cuda.current_stream().cuda_stream
    d, F = 4096, 14336
    x = torch.randn(F, device="cuda")
    nw = torch.ones(F, device="cuda")
    res = {}
    for name, t, R, K, epi, norm in [("gateup", Q4_K, 2 * F, d, 2, True), ("down_q4k", Q4_K, d, F, 1, False),
                                     ("down_q6k", Q6_K, d, F, 1, False), ("wo", Q4_K, d, d, 1, False),
                                     ("lmhead", Q6_K, 128256, d, 0, True)]:
        nb = hip.qbytes(t, R, K)
        ncopy = max(2, (700 << 20) // nb + 1)
        ws = []
        for c in range(ncopy):
            b = torch.empty(nb, dtype=torch.uint8, device="cuda")
            hip.fill_random(b.data_ptr(), t, R, K, 0.02, c + 1, s)
            ws.append(b)
        n_out = R // 2 if epi == 2 else R
        out = torch.zeros(n_out, device="cuda")
        clk = torch.zeros(4096 * 5, dtype=torch.int64, device="cuda")
        for c in range(ncopy):  # warm-up (and evicts the copy timed last from the caches)
            hip.gemv(ws[c].data_ptr(), t, R, K, x.data_ptr(), nw.data_ptr() if norm else 0, 1e-5, out.data_ptr(),
                     n_out, epi, s, dbg_clk=clk.data_ptr())
        torch.cuda.synchronize()
        clk.zero_()
        hip.gemv(ws[0].data_ptr(), t, R, K, x.data_ptr(), nw.data_ptr() if norm else 0, 1e-5, out.data_ptr(),
                 n_out, epi, s, dbg_clk=clk.data_ptr())
        torch.cuda.synchronize()
        a = clk.view(-1, 5).cpu().numpy()
        a = a[a[:, 0] > 0]
        base = a[:, 0].min()
        us = lambda v: np.round((v - base) / 100.0, 2)  # 100 MHz wall clock
        ent, pro, first, ext = us(a[:, 0]), us(a[:, 1]), us(a[:, 2]), us(a[:, 3])
        pct = lambda v: [float(np.percentile(v, p)) for p in (0, 50, 90, 100)]
        res[name] = {"blocks": int(len(a)), "MB": round(nb / 1e6, 1), "total_us": float(ext.max()),
                     "entry_p0_50_90_100": pct(ent), "prologue_end": pct(pro), "first_item_end": pct(first),
                     "exit": pct(ext), "items_w0": pct(a[:, 4]),
                     "eff_TB_s": round(nb / (ext.max() * 1e-6) / 1e12, 2)}
        del ws
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
