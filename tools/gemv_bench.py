"""Per-kernel timing of the decode kernels at Llama-3-8B shapes (1 GPU).

Each kernel is captured N times back to back into a torch CUDA graph (so the
number includes one graph kernel boundary, as in the engine's decode step) and
the replay is timed; bandwidth = weight bytes / time.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

Q4_K, Q5_K, Q6_K, Q8_0 = 12, 13, 14, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default="")
    ap.add_argument("--eager", action="store_true", help="plain launches (for rocprofv3 kernel traces)")
    ap.add_argument("--debug", action="store_true", help="also time kernel prefixes (stage breakdown)")
    args = ap.parse_args()
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    s = torch.cuda.current_stream().cuda_stream
    res = {}

    def timed(name, fn, nbytes):
        if args.only and args.only not in name:
            return
        if args.eager:
            for _ in range(args.reps):
                fn()
            torch.cuda.synchronize()
            return
        g = torch.cuda.CUDAGraph()
        fn()
        torch.cuda.synchronize()
        cs = torch.cuda.Stream()
        with torch.cuda.stream(cs):
            with torch.cuda.graph(g):
                for _ in range(args.reps):
                    fn(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (5 * args.reps)
        res[name] = {"us": round(us, 2), "TB_s": round(nbytes / us / 1e6, 2)}

    def mat(t, R, K, seed):
        nb = hip.qbytes(t, R, K)
        buf = torch.empty(nb, dtype=torch.uint8, device="cuda")
        hip.fill_random(buf.data_ptr(), t, R, K, 0.02, seed, s)
        return buf, nb

    d, F, V = 4096, 14336, 128256
    x = torch.randn(F, device="cuda")
    nw = torch.ones(F, device="cuda")
    out = torch.zeros(2 * F, device="cuda")
    bufs = []
    # weights are cycled through enough copies (>= 600 MB) that every launch streams
    # from HBM, as in a real decode step (a single re-read matrix would sit in the
    # 256 MB infinity cache and flatter the kernel)
    def copies(nb):
        return max(1, min(32, (600 << 20) // nb + 1))

    for name, t, R, K, epi, norm in [
        ("wo_q4k_4096x4096_add", Q4_K, d, d, 1, False),
        ("gateup_q4k_28672x4096_swiglu", Q4_K, 2 * F, d, 2, True),
        ("down_q4k_4096x14336_add", Q4_K, d, F, 1, False),
        ("down_q6k_4096x14336_add", Q6_K, d, F, 1, False),
        ("lmhead_q6k_128256x4096", Q6_K, V, d, 0, True),
        ("wq_q4k_4096x4096_norm", Q4_K, d, d, 0, True),
        ("wv_q6k_1024x4096_norm", Q6_K, 1024, d, 0, True),
    ]:
        if args.only and args.only not in name:
            continue
        nb = hip.qbytes(t, R, K)
        ws = [mat(t, R, K, 1000 * len(bufs) + c + 1)[0] for c in range(copies(nb))]
        bufs.append(ws[0])
        n_out = R // 2 if epi == 2 else R
        big_out = torch.zeros(n_out, device="cuda")
        ctr = [0]

        for dbg in ((0, 1, 2, 3) if args.debug else (0,)):
            def fn(st=s, ws=ws, t=t, R=R, K=K, epi=epi, norm=norm, n_out=n_out, big_out=big_out, dbg=dbg, ctr=ctr):
                w = ws[ctr[0] % len(ws)]
                ctr[0] += 1
                hip.gemv(w.data_ptr(), t, R, K, x.data_ptr(), nw.data_ptr() if norm else 0, 1e-5, big_out.data_ptr(),
                         n_out, epi, st, debug=dbg)
            timed(name + ("" if dbg == 0 else f"_dbg{dbg}"), fn, nb)
        del ws[1:]

    # fused QKV + RoPE + KV append (Q/K Q4_K, V Q6_K as in the bumped layers; and all-Q4_K)
    n_ctx, hd = 1024, 128
    kc = torch.zeros(8, n_ctx, hd, dtype=torch.float16, device="cuda")
    vc = torch.zeros_like(kc)
    q = torch.zeros(d, device="cuda")
    pos = torch.tensor([500], dtype=torch.int32, device="cuda")
    rope = torch.randn(n_ctx * hd // 2 * 2, device="cuda")
    NC = 32
    wqs = [mat(Q4_K, d, d, 100 + c)[0] for c in range(NC)]
    wks = [mat(Q4_K, 1024, d, 200 + c)[0] for c in range(NC)]
    wv4s = [mat(Q4_K, 1024, d, 300 + c)[0] for c in range(NC)]
    wv6s = [mat(Q6_K, 1024, d, 400 + c)[0] for c in range(NC)]
    nq_b, nk_b = hip.qbytes(Q4_K, d, d), hip.qbytes(Q4_K, 1024, d)
    nv4, nv6 = hip.qbytes(Q4_K, 1024, d), hip.qbytes(Q6_K, 1024, d)
    qctr = [0]
    for name, wvs, tv, nvb in [("qkv_q4k_all", wv4s, Q4_K, nv4), ("qkv_q4k_v_q6k", wv6s, Q6_K, nv6)]:
        def fn(st=s, wvs=wvs, tv=tv):
            c = qctr[0] % NC
            qctr[0] += 1
            hip.gemv_qkv(wqs[c].data_ptr(), Q4_K, wks[c].data_ptr(), Q4_K, wvs[c].data_ptr(), tv, d, 1024, d,
                         x.data_ptr(), nw.data_ptr(), 1e-5, q.data_ptr(), kc.data_ptr(), vc.data_ptr(), n_ctx, hd,
                         pos.data_ptr(), rope.data_ptr(), st)
        timed(name, fn, nq_b + nk_b + nvb)
    del wqs, wks, wv4s, wv6s

    # decode attention, 32 q heads on 8 kv heads, hd 128, at a few KV lengths
    part = torch.empty(hip.attn_decode_workspace_floats(n_ctx, 32, hd), device="cuda")
    cnt = torch.zeros(64, dtype=torch.int32, device="cuda")
    qa = torch.randn(32 * hd, device="cuda")
    ao = torch.zeros(32 * hd, device="cuda")
    kc.normal_()
    vc.normal_()
    for L in (128, 512, 1000):
        p = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
        for stop in ((0, 1, 2, 3, 4) if args.debug else (0,)):
            def fn(st=s, p=p, stop=stop):
                hip.attn_decode(qa.data_ptr(), kc.data_ptr(), vc.data_ptr(), p.data_ptr(), n_ctx, 32, 8, hd,
                                hd ** -0.5, part.data_ptr(), ao.data_ptr(), st, cnt.data_ptr(), debug_stop=stop)
            timed(f"attn_decode_L{L}" + ("" if stop == 0 else f"_stop{stop}"), fn, 2 * 8 * L * hd * 2)
    # in-kernel timeline (wall_clock64 ticks of 10 ns) of block (0,0) and the merging block
    stamps = torch.zeros(16 * 8 * ((n_ctx + 63) // 64), dtype=torch.int64, device="cuda")
    for L in (128, 1000):
        p = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
        for _ in range(3):
            hip.attn_decode(qa.data_ptr(), kc.data_ptr(), vc.data_ptr(), p.data_ptr(), n_ctx, 32, 8, hd, hd ** -0.5,
                            part.data_ptr(), ao.data_ptr(), s, cnt.data_ptr(), dbg_clk=stamps.data_ptr())
        torch.cuda.synchronize()
        st0 = stamps.tolist()[:16]   # block (0, 0): absolute stamps -> us after its entry
        res[f"attn_timeline_L{L}_us"] = {"us": [round((v - st0[0]) / 100.0, 2) if v else None for v in st0[1:11]],
                                        "TB_s": 0}
    # floor: an empty kernel (debug_stop=1 at L=1 exits immediately in every block)
    p1 = torch.tensor([0], dtype=torch.int32, device="cuda")
    timed("empty_kernel_floor", lambda st=s: hip.attn_decode(qa.data_ptr(), kc.data_ptr(), vc.data_ptr(),
          p1.data_ptr(), n_ctx, 32, 8, hd, 1.0, part.data_ptr(), ao.data_ptr(), st, cnt.data_ptr(), debug_stop=1), 1)
    # shader clock: alone, and right behind a heavy GEMV in the same stream
    clk = torch.zeros(3, dtype=torch.int64, device="cuda")
    for label, pre in (("alone", None), ("after_gemv", bufs[1] if len(bufs) > 1 else None)):
        vals = []
        for _ in range(5):
            if pre is not None:
                hip.gemv(pre.data_ptr(), Q4_K, 2 * F, d, x.data_ptr(), nw.data_ptr(), 1e-5, out.data_ptr(), F, 2, s)
            hip.clock_probe(clk.data_ptr(), 20000, s)
            torch.cuda.synchronize()
            c, w = clk[0].item(), clk[1].item()
            vals.append(c / (w / 100.0))   # cycles per us = MHz (wall clock 100 MHz)
        res[f"shader_MHz_{label}"] = {"us": round(sum(vals) / len(vals), 1), "TB_s": 0}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
