"""Back-to-back timeline of one decode GEMV shape: N instrumented launches in a
row (eager or captured in a graph), weights cycled through HBM-resident copies.
Reports per launch the first-entry / last-exit wall-clock stamps, so the gap
between one launch's last block and the next launch's first block (the kernel
boundary) and each launch's in-kernel span can be read separately."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

Q4_K, Q6_K = 12, 14


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--graph", action="store_true")
    args = ap.parse_args()
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    s = torch.cuda.current_stream().cuda_stream
    d, F = 4096, 14336
    x = torch.randn(F, device="cuda")
    nw = torch.ones(F, device="cuda")
    res = {}
    for name, t, R, K, epi, norm in [("gateup", Q4_K, 2 * F, d, 2, True), ("wo", Q4_K, d, d, 1, False),
                                     ("down_q6k", Q6_K, d, F, 1, False)]:
        nb = hip.qbytes(t, R, K)
        ncopy = max(2, (700 << 20) // nb + 1)
        ws = []
        for c in range(ncopy):
            b = torch.empty(nb, dtype=torch.uint8, device="cuda")
            hip.fill_random(b.data_ptr(), t, R, K, 0.02, c + 1, s)
            ws.append(b)
        n_out = R // 2 if epi == 2 else R
        out = torch.zeros(n_out, device="cuda")
        clks = [torch.zeros(4096 * 5, dtype=torch.int64, device="cuda") for _ in range(args.n)]

        def run(st):
            for i in range(args.n):
                hip.gemv(ws[i % ncopy].data_ptr(), t, R, K, x.data_ptr(), nw.data_ptr() if norm else 0, 1e-5,
                         out.data_ptr(), n_out, epi, st, dbg_clk=clks[i].data_ptr())
        run(s)
        torch.cuda.synchronize()
        if args.graph:
            g = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream()
            with torch.cuda.stream(cs):
                with torch.cuda.graph(g):
                    run(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            for c in clks:
                c.zero_()
            g.replay()
        else:
            for c in clks:
                c.zero_()
            run(s)
        torch.cuda.synchronize()
        spans = []
        base = None
        for c in clks:
            a = c.view(-1, 5).cpu().numpy()
            a = a[a[:, 0] > 0]
            if base is None:
                base = a[:, 0].min()
            spans.append(((a[:, 0].min() - base) / 100.0, (np.median(a[:, 1]) - base) / 100.0,
                          (a[:, 3].max() - base) / 100.0))
        per = [{"entry": round(e, 2), "pro_med": round(p, 2), "exit": round(x_, 2)} for e, p, x_ in spans]
        gaps = [round(spans[i + 1][0] - spans[i][2], 2) for i in range(len(spans) - 1)]
        body = [round(x_ - e, 2) for e, _, x_ in spans]
        res[name] = {"MB": round(nb / 1e6, 1), "per_launch_us": round((spans[-1][2] - spans[0][0]) / len(spans), 2),
                     "gaps": gaps, "body": body, "launches": per}
        del ws
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
