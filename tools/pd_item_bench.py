"""Cycles per ring item of the persistent decode consumer code, alone (no loader, no
hand-offs): one workgroup per CU, every consumer wave loops over the same LDS item."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    out = torch.zeros(256 * 8, dtype=torch.int64, device="cuda")
    res = {}
    for name, t, rows, K in [("q4k_6rows_K4096", 12, 6, 4096), ("q4k_1row_K14336", 12, 1, 14336),
                             ("q6k_4rows_K4096", 14, 4, 4096), ("q6k_1row_K14336", 14, 1, 14336),
                             ("q8_0_3rows_K4096", 8, 3, 4096)]:
        for blocks in (1, 256):
            hip.pd_item_bench(t, rows, K, 2000, blocks, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            v = out.view(256, 8)[:blocks, :6].float()
            res[f"{name}_blocks{blocks}"] = [round(float(v.median()), 1), round(float(v.max()), 1)]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
