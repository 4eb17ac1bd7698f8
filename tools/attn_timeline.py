"""Batched decode attention (continuous batching rows) timeline from per-block wall_clock64
stamps (attention.hip TL instantiation): when the blocks start, how long the K/V loads, the
partial store, the split counter and the last-arriver merge take - for B rows at KV length L.

    python tools/attn_timeline.py [--rows 6] [--L 700]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6)
    ap.add_argument("--L", type=int, default=700)
    ap.add_argument("--n-ctx", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch
    from gpu_helpers import hip, stream
    h = hip()
    B, L, n_ctx, H, KV, hd = args.rows, args.L, args.n_ctx, 32, 8, 128
    slot_stride = KV * n_ctx * hd
    kc = torch.randn(B * slot_stride, device="cuda").half()
    vc = torch.randn(B * slot_stride, device="cuda").half()
    q = torch.randn(B, H * hd, device="cuda")
    out = torch.zeros(B, H * hd, device="cuda")
    outh = torch.zeros(B, H * hd, dtype=torch.float16, device="cuda")
    part = torch.empty(B * h.attn_decode_workspace_floats(n_ctx, H, hd), device="cuda")
    cnt = torch.zeros(64 * B, dtype=torch.int32, device="cuda")
    pos = torch.full((B,), L - 1, dtype=torch.int32, device="cuda")
    slots = torch.arange(B, dtype=torch.int32, device="cuda")
    nsplit = (n_ctx + 63) // 64
    clk = torch.zeros(16 * KV * nsplit * B, dtype=torch.int64, device="cuda")

    def run(dbg):
        h.attn_decode(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), pos.data_ptr(), n_ctx, H, KV, hd, hd ** -0.5,
                      part.data_ptr(), out.data_ptr(), stream(), cnt.data_ptr(), dbg_clk=dbg, batch=B,
                      slots=slots.data_ptr(), slot_stride=slot_stride, out_h=outh.data_ptr())
    run(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        with torch.cuda.graph(g):
            for _ in range(args.reps):
                h.attn_decode(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), pos.data_ptr(), n_ctx, H, KV, hd,
                              hd ** -0.5, part.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream,
                              cnt.data_ptr(), batch=B, slots=slots.data_ptr(), slot_stride=slot_stride,
                              out_h=outh.data_ptr())
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) * 1e3 / args.reps
    run(clk.data_ptr())
    torch.cuda.synchronize()
    c = clk.view(-1, 16).cpu().numpy()
    c = c[c[:, 0] > 0]
    t0 = c[:, 0].min()
    act = c[c[:, 2] > 0]   # blocks that did work (start < L)

    def q_(v):
        v = np.sort(v)
        return [round(float(v[len(v) // 2]) / 100, 2), round(float(v[int(len(v) * .9)]) / 100, 2),
                round(float(v[-1]) / 100, 2)]
    res = {"B": B, "L": L, "graph_us_per_launch": round(per, 2), "blocks": int(len(c)), "active": int(len(act)),
           "span_us": round(float(c[:, 9].max() - t0) / 100 if (c[:, 9] > 0).any() else 0, 2),
           "start_p50_p90_max": q_(act[:, 0] - t0),
           "loads_issued_p50_p90_max": q_(act[:, 1] - act[:, 0]),
           "v_staged": q_(act[:, 2] - act[:, 0]),
           "partials_met": q_(act[:, 4] - act[:, 0]),
           "partial_stored": q_(act[:, 5] - act[:, 0]),
           "counter_taken": q_(act[:, 6] - act[:, 0])}
    m = c[c[:, 8] > 0]
    if len(m):
        res["merge_start_after_kernel_start"] = q_(m[:, 8] - t0)
        res["merge_dur"] = q_(m[:, 9] - m[:, 8])
        res["merge_end_after_kernel_start"] = q_(m[:, 9] - t0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
