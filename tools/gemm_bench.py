"""Prefill GEMM timing at Llama-3-8B shapes (1 GPU): Y[T][N] = X[T][K] . W^T.

Weights are random planar blocks (hip.fill_random); the number is the mean over
--reps back-to-back launches (events around the batch) and TFLOP/s = 2*T*N*K / time.
--eager only launches (for rocprofv3 --pmc passes).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

Q4_K, Q6_K = 12, 14
STORE, ADD, SWIGLU = 0, 1, 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--t16", action="store_true", help="the tile16 prefill GEMM (gemm_t16, f16 X)")
    ap.add_argument("--cfg", default="", help="gemm_t16 block shape 'waves,tokens' (8,128 / 8,64 / 4,64)")
    args = ap.parse_args()
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    s = torch.cuda.current_stream().cuda_stream
    d, F, T = 4096, 14336, args.T
    res = {"T": T, "kernel": "gemm_t16" if args.t16 else "gemm_dq", "cfg": args.cfg}
    cfg = 0
    if args.cfg:
        nw, tm = (int(v) for v in args.cfg.split(","))
        cfg = nw * 1000 + tm
    for name, t, R, K, epi in [
        ("gateup_q4k_swiglu", Q4_K, 2 * F, d, SWIGLU),
        ("down_q4k_add", Q4_K, d, F, ADD),
        ("down_q6k_add", Q6_K, d, F, ADD),
        ("wq_q4k_store", Q4_K, d, d, STORE),
        ("wo_q4k_add", Q4_K, d, d, ADD),
    ]:
        if args.only and args.only not in name:
            continue
        w = torch.empty(hip.qbytes(t, R, K), dtype=torch.uint8, device="cuda")
        hip.fill_random(w.data_ptr(), t, R, K, 0.02, 7, s)
        x = torch.randn(T, K, device="cuda").to(torch.float16 if args.t16 else torch.bfloat16)
        out = torch.zeros(T, R, device="cuda")
        ob = torch.zeros(T, R // 2, device="cuda", dtype=torch.bfloat16)
        if args.t16:
            tw = torch.empty(hip.t16_bytes(t, R, K), dtype=torch.uint8, device="cuda")
            hip.t16_repack(w.data_ptr(), t, R, K, tw.data_ptr(), s, epi == SWIGLU)

        def fn():
            if args.t16:
                hip.gemm_t16(tw.data_ptr(), t, R, K, x.data_ptr(), T, out.data_ptr(), R, ob.data_ptr(), R // 2, epi, s, cfg=cfg)
            else:
                hip.gemm(w.data_ptr(), t, R, K, x.data_ptr(), T, out.data_ptr(), ob.data_ptr(), R, epi, s)

        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if args.eager:
            continue
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        res[name] = {"us": round(us, 1), "TFLOPs": round(2.0 * T * R * K / us / 1e6, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
