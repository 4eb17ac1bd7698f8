"""Per-block timeline of single bmm launches (the batched decode projections) from the
kernel's wall_clock64 stamps (BmmArgs::dbg_clk, 100 MHz): when blocks start after the first
one, how long the weight issue / x staging / first tile / whole block take. Tells a latency
floor (every block short, kernel long: dispatch) from a stream (blocks long) from a tail.

    python tools/bmm_timeline.py [--rows 6] [--shapes wq,wk,down,gate_up_sw]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"gate_up_sw": (12, 28672, 4096), "down": (12, 4096, 14336), "down6": (14, 4096, 14336),
          "wq": (12, 4096, 4096), "wk": (12, 1024, 4096), "wv6": (14, 1024, 4096), "head": (14, 128256, 4096)}


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6)
    ap.add_argument("--shapes", default="wk,wq,down,gate_up_sw,down6,wv6")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch
    from gpu_helpers import hip, stream
    h = hip()
    B = args.rows
    res = {}
    for name in args.shapes.split(","):
        t, R, K = SHAPES[name]
        nbytes = h.t16_bytes(t, R, K)
        nbuf = max(2, min(8, (600 << 20) // nbytes + 1))
        ws = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(nbuf)]  # random tile16 bytes
        xh = torch.randn(16, K, device="cuda").half()
        out = torch.zeros(16, R, device="cuda")
        hout = torch.zeros(16, R // 2, dtype=torch.float16, device="cuda")
        clk = torch.zeros(8192 * 8, dtype=torch.int64, device="cuda")
        sw = name.endswith("_sw")
        durs, rows = [], []
        for i in range(args.reps):
            clk.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h.bmm(ws[i % nbuf].data_ptr(), t, R, K, xh.data_ptr(), K, out.data_ptr(), R, B, stream(),
                  h_out=hout.data_ptr() if sw else 0, ldh_out=R // 2, dbg_clk=clk.data_ptr())
            e1.record()
            torch.cuda.synchronize()
            durs.append(e0.elapsed_time(e1) * 1e3)
            c = clk.view(-1, 8).cpu().numpy()
            c = c[c[:, 0] > 0]
            rows.append(c)
        c = rows[-1]
        t0 = c[:, 0].min()
        us = lambda x: (x / 100.0)  # noqa: E731  (100 MHz ticks -> us)
        start = us(c[:, 0] - t0)
        issue = us(c[:, 1] - c[:, 0])
        staged = us(c[:, 2] - c[:, 0])
        first = us(np.where(c[:, 3] > 0, c[:, 3] - c[:, 0], 0))
        life = us(c[:, 4] - c[:, 0])
        end = us(c[:, 4] - t0)
        r = {"blocks": int(len(c)), "event_us": round(float(np.median(durs)), 2),
             "span_us": round(float(end.max()), 2),
             "start_us_p50_p100": [round(float(pct(start, .5)), 2), round(float(start.max()), 2)],
             "x_staged_us_p50_p90": [round(float(pct(staged, .5)), 2), round(float(pct(staged, .9)), 2)],
             "first_tile_us_p50_p90": [round(float(pct(first, .5)), 2), round(float(pct(first, .9)), 2)],
             "block_life_us_p50_p90_max": [round(float(pct(life, .5)), 2), round(float(pct(life, .9)), 2),
                                           round(float(life.max()), 2)],
             "tiles_per_block": [int(c[:, 5].min()), int(c[:, 5].max())],
             "TBps": round(nbytes / (np.median(durs) * 1e-6) / 1e12, 2)}
        res[name] = r
        print(name, json.dumps(r), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
