"""MFMA batched-projection microbenchmark: one bmm launch per 8B projection shape at B rows
(HIP events; weights are random bytes - timing only). Distinct weight buffers rotate so a
shape is not re-read from the 256 MB memory-side cache."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rows", default="1,8,16")
    ap.add_argument("--debug", type=int, default=0)
    args = ap.parse_args()
    import torch
    from gpu_helpers import hip, stream
    from llama_fastapi_k8s_gpu_amd.gguf.constants import GGMLType
    h = hip()
    shapes = [("gate_up", GGMLType.Q4_K, 28672, 4096), ("gate_up_sw", GGMLType.Q4_K, 28672, 4096),
              ("down", GGMLType.Q4_K, 4096, 14336),
              ("down6", GGMLType.Q6_K, 4096, 14336), ("wq", GGMLType.Q4_K, 4096, 4096),
              ("wk", GGMLType.Q4_K, 1024, 4096), ("head", GGMLType.Q6_K, 128256, 4096)]
    res = {}
    for name, t, R, K in shapes:
        nbytes = h.t16_bytes(int(t), R, K)
        nbuf = max(2, min(8, (600 << 20) // nbytes + 1))
        ws = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(nbuf)]
        xh = torch.randn(16, K, device="cuda").half()
        out = torch.zeros(16, R, device="cuda")
        hout = torch.zeros(16, R // 2, dtype=torch.float16, device="cuda")
        sw = name.endswith("_sw")  # SwiGLU epilogue (one K part, f16 output)
        for B in [int(b) for b in args.rows.split(",")]:
            def fn(i):
                h.bmm(ws[i % nbuf].data_ptr(), int(t), R, K, xh.data_ptr(), K, out.data_ptr(), R, B, stream(),
                      debug=args.debug, h_out=hout.data_ptr() if sw else 0, ldh_out=R // 2)
            fn(0)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(args.reps):
                fn(i + 1)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            res[f"{name}_B{B}_us"] = round(us, 2)
            res[f"{name}_B{B}_TBps"] = round(nbytes / (us * 1e-6) / 1e12, 2)
        del ws
    print(json.dumps(res))


if __name__ == "__main__":
    main()
