"""GPU sampler timing at V = 128256 (Llama-3): graph-replayed time per sample()
(3 kernels) and the stage-2 in-kernel timeline."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from llama_fastapi_k8s_gpu_amd.runtime import load_hip
    h = load_hip()
    V = 128256
    rng = np.random.default_rng(0)
    dl = torch.from_numpy((rng.standard_normal(V) * 3).astype(np.float32)).cuda()
    pb = np.frombuffer(h.sampler_params_bytes(40, 0.9, 0.05, 1.2, 1.1, 0.7, 0.8, 64, 7, 0), np.uint8)
    dp = torch.from_numpy(pb.copy()).cuda()
    ring = torch.from_numpy(rng.integers(0, V, 64).astype(np.int32)).cuda()
    st = torch.from_numpy(np.array([0, 0, 0, 64, 0, 0, 0, 0], np.int32)).cuda()
    cand = torch.zeros(h.sampler_cand_words(V), dtype=torch.int32, device="cuda")
    clk = torch.zeros(8, dtype=torch.int64, device="cuda")

    def run(s, dbg=0):
        h.sample(dl.data_ptr(), V, dp.data_ptr(), ring.data_ptr(), st.data_ptr(), cand.data_ptr(), 0, 0,
                 0, s, dbg_clk=dbg)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        run(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        with torch.cuda.graph(g):
            for _ in range(50):
                run(torch.cuda.current_stream().cuda_stream)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    res = {"sample_us_graph": round(e0.elapsed_time(e1) * 1e3 / 200, 2)}
    run(s, clk.data_ptr())
    torch.cuda.synchronize()
    res["stage2_timeline_us"] = [round(v / 100.0, 2) for v in clk.tolist()[:4]]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
