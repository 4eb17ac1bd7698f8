"""Kernel-boundary cost of the batched decode projections (bmm.hip wave-owned kernels) in graph
chains of their own: per XCD, the gap from the last block's exit stamp of launch k to the first
block's entry stamp of launch k + 1 (wall_clock64 is per XCD, so gaps are taken within one XCD),
the span of each launch on each XCD, and the chain's event time per launch.

Chains: Wo (split-K, fp32 atomics into the residual), gate/up (SwiGLU f16 store epilogue), down
(split-K atomics, K = 14336), and the three alternating as in a layer. Weights are random tile16
bytes rotated over enough buffers to defeat the L2 / Infinity Cache (as a real step streams them).
Each chain runs in three forms (BmmArgs::debug): the full kernel (0), the kernel without its
epilogue writes (3), and the bare launch that exits at entry (2) - which part of a boundary the
launch shape, the weight stream and the epilogue's writes each account for.

    python tools/boundary_bench.py [--rows 6] [--n 24] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"wo": (12, 4096, 4096, False), "gu": (12, 28672, 4096, True), "down": (12, 4096, 14336, False)}


def per_xcd(c):
    """{xcc: (first entry, last exit)} of one launch's stamps [blocks, 8]."""
    c = c[c[:, 0] > 0]
    out = {}
    for x in range(16):
        m = (c[:, 6] & 0xF) == x
        if m.any():
            out[x] = (int(c[m, 0].min()), int(c[m, 4].max()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6)
    ap.add_argument("--n", type=int, default=24, help="launches per chain")
    ap.add_argument("--json", default=None)
    ap.add_argument("--debug", default="0,3,2", help="BmmArgs::debug forms to run (wave-owned kernels: "
                    "0 full, 2 exit at entry, 3 no epilogue writes, 4 weight stream only, 5 x staging + "
                    "weights, 6 weights + MFMA)")
    ap.add_argument("--norm", action="store_true", help="gate/up stages f32 x rows with the RMSNorm folded "
                    "(as the engine's batched step does)")
    ap.add_argument("--chains", default="wo,gu,down,layer")
    args = ap.parse_args()
    import numpy as np
    import torch
    from gpu_helpers import hip
    h = hip()
    B = args.rows
    bufs = {}
    for name, (t, R, K, _) in SHAPES.items():
        nb = h.t16_bytes(t, R, K)
        bufs[name] = [torch.randint(0, 255, (nb,), dtype=torch.uint8, device="cuda")
                      for _ in range(max(2, (320 << 20) // nb + 1))]
    xh = torch.randn(16, 14336, device="cuda").half()
    out = torch.zeros(16, 28672, device="cuda")
    hout = torch.zeros(16, 14336, dtype=torch.float16, device="cuda")
    xf = torch.randn(16, 4096, device="cuda")
    nw = torch.ones(4096, device="cuda")
    chains = {"wo": ["wo"] * args.n, "gu": ["gu"] * args.n, "down": ["down"] * args.n,
              "layer": (["wo", "gu", "down"] * args.n)[:args.n]}
    chains = {k: v for k, v in chains.items() if k in args.chains.split(",")}
    res = {"env": {k: os.environ.get(k) for k in ("HIP_FORCE_DEV_KERNARG", "GPU_MAX_HW_QUEUES")},
           "norm": args.norm}
    for dbg, (cname, seq) in [(int(d), c) for d in args.debug.split(",") for c in chains.items()]:
        clk = torch.zeros(len(seq), 8192 * 8, dtype=torch.int64, device="cuda")
        use = {k: 0 for k in SHAPES}

        def run(st):
            for i, name in enumerate(seq):
                t, R, K, sw = SHAPES[name]
                w = bufs[name][use[name] % len(bufs[name])]
                use[name] += 1
                nx = sw and args.norm
                h.bmm(w.data_ptr(), t, R, K, xh.data_ptr(), K, out.data_ptr(), R, B, st, debug=dbg,
                      h_out=hout.data_ptr() if sw else 0, ldh_out=R // 2, dbg_clk=clk[i].data_ptr(),
                      xf=xf.data_ptr() if nx else 0, ldxf=K if nx else 0, norm=nw.data_ptr() if nx else 0,
                      eps=1e-5)
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        with torch.cuda.stream(cs):
            run(cs.cuda_stream)
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                run(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        times = []
        for _ in range(4):
            clk.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / len(seq))
        c = clk.view(len(seq), -1, 8).cpu().numpy()
        px = [per_xcd(c[i]) for i in range(len(seq))]
        gaps, spans = {}, {}
        for i in range(len(seq)):
            for x, (s0, s1) in px[i].items():
                spans.setdefault(seq[i], []).append((s1 - s0) / 100.0)
                if i + 1 < len(seq) and x in px[i + 1]:
                    gaps.setdefault(f"{seq[i]}->{seq[i + 1]}", []).append((px[i + 1][x][0] - s1) / 100.0)
        r = {"us_per_launch_event": round(float(np.median(times)), 2),
             "span_us_p50": {k: round(float(np.median(v)), 2) for k, v in spans.items()},
             "gap_us_p50_p90": {k: [round(float(np.median(v)), 2), round(float(np.percentile(v, 90)), 2)]
                                for k, v in gaps.items()}}
        res[f"{cname}_debug{dbg}"] = r
        print(f"{cname} debug={dbg}", json.dumps(r), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
