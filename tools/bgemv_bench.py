"""Batched-GEMV microbenchmark: one launch of each 8B projection shape at NB rows, full
kernel vs no prologue math (debug 1) vs loads only (debug 2), timed with HIP events."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rows", default="1,2,4,8")
    args = ap.parse_args()
    import torch
    from gpu_helpers import hip, stream
    from llama_fastapi_k8s_gpu_amd.gguf.constants import GGMLType
    h = hip()
    shapes = [("gate_up", GGMLType.Q4_K, 28672, 4096), ("down", GGMLType.Q4_K, 4096, 14336),
              ("wq", GGMLType.Q4_K, 4096, 4096), ("head", GGMLType.Q6_K, 128256, 4096)]
    res = {}
    for name, t, R, K in shapes:
        nbytes = h.qbytes(int(t), R, K)
        w = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
        # sane f16 scales are not needed for timing; outputs are discarded
        x = torch.randn(8, 2 * K, device="cuda")
        out = torch.zeros(8, R, device="cuda")
        for B in [int(b) for b in args.rows.split(",")]:
            for dbg in (0, 1, 2):
                fn = lambda: h.bgemv(w.data_ptr(), int(t), R, K, x.data_ptr(), 2 * K, name == "down", 0, 1e-5,
                                     out.data_ptr(), R, B, stream(), debug=dbg)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.reps
                res[f"{name}_B{B}_d{dbg}_us"] = round(us, 2)
            res[f"{name}_B{B}_GBps"] = round(nbytes / (res[f"{name}_B{B}_d0_us"] * 1e-6) / 1e9, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
