"""Fused decode FFN (ffn_fused.hip) at Llama-3-8B shapes: N launches back to back
in a graph (weights cycled through HBM-resident copies), per-workgroup stamps:
entry, prologue done, phase A done, published, waits done, h in LDS, exit.
Compare per_launch_us with the unfused gate/up + down pair (gemv_chain_timeline)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

Q4_K, Q6_K = 12, 14
STAGES = ["entry", "prologue", "phaseA", "published", "waited", "h_lds", "exit"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--down", default="q6k")
    args = ap.parse_args()
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    s = torch.cuda.current_stream().cuda_stream
    d, F = 4096, 14336
    tdn = Q6_K if args.down == "q6k" else Q4_K
    ngu, ndn = hip.qbytes(Q4_K, 2 * F, d), hip.qbytes(tdn, d, F)
    ncopy = max(2, (900 << 20) // (ngu + ndn) + 1)
    gus, dns = [], []
    for c in range(ncopy):
        g = torch.empty(ngu, dtype=torch.uint8, device="cuda")
        hip.fill_random(g.data_ptr(), Q4_K, 2 * F, d, 0.02, 2 * c + 1, s)
        dn = torch.empty(ndn, dtype=torch.uint8, device="cuda")
        hip.fill_random(dn.data_ptr(), tdn, d, F, 0.02, 2 * c + 2, s)
        gus.append(g)
        dns.append(dn)
    x = torch.randn(d, device="cuda")
    nw = torch.ones(d, device="cuda")
    h = torch.zeros(F, device="cuda")
    ctr = torch.zeros(2, 32, dtype=torch.int32, device="cuda")
    err = torch.zeros(4, dtype=torch.int32, device="cuda")
    clks = [torch.zeros(1024 * 8, dtype=torch.int64, device="cuda") for _ in range(args.n)]

    def run(st, stamp=True):
        for i in range(args.n):
            hip.ffn_fused(gus[i % ncopy].data_ptr(), Q4_K, dns[i % ncopy].data_ptr(), tdn, d, F, x.data_ptr(),
                          nw.data_ptr(), 1e-5, h.data_ptr(), ctr[i % 2].data_ptr(), ctr[(i + 1) % 2].data_ptr(),
                          err.data_ptr(), st, dbg_clk=clks[i].data_ptr() if stamp else 0)
    res = {}
    for stamp in (False, True):
        run(s, stamp)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        with torch.cuda.stream(cs):
            with torch.cuda.graph(g):
                run(torch.cuda.current_stream().cuda_stream, stamp)
        torch.cuda.synchronize()
        for c in clks:
            c.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        res["per_launch_us_graph" + ("_stamped" if stamp else "")] = round(e0.elapsed_time(e1) * 1e3 / args.n, 2)
    res["err"] = int(err[0].item())
    per = []
    for c in clks:
        a = c.view(-1, 8).cpu().numpy()
        a = a[a[:, 0] > 0]
        base = a[:, 0].min()
        row = {}
        for k, nm in enumerate(STAGES):
            v = a[:, k]
            v = v[v > 0]
            if len(v):
                row[nm] = [round(float(np.percentile((v - base) / 100.0, p)), 2) for p in (0, 50, 90, 100)]
        per.append(row)
    res["stages_p0_50_90_100_us"] = per[len(per) // 2]
    res["MB"] = round((ngu + ndn) / 1e6, 1)
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
