"""Per-launch cost of a workgroup shape: graph chains of a trivial kernel at
256 / 512 / 1024 threads per block, with and without an 80 KiB LDS request."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    hip = load_hip()
    out = torch.zeros(1024, device="cuda")
    res = {}
    N = 100
    for threads, blocks, lds, iters in [(256, 1024, 0, 0), (256, 256, 0, 0), (512, 512, 0, 0), (1024, 256, 0, 0),
                                        (1024, 256, 82 * 1024, 0), (256, 1024, 0, 2000), (1024, 256, 0, 2000),
                                        (1024, 256, 82 * 1024, 2000)]:
        def run(st):
            for _ in range(N):
                hip.launch_probe(threads, blocks, lds, iters, out.data_ptr(), st)
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        with torch.cuda.stream(cs):
            run(cs.cuda_stream)
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                run(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[f"t{threads}_b{blocks}_lds{lds // 1024}k_it{iters}"] = round(e0.elapsed_time(e1) * 1e3 / (3 * N), 3)
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
