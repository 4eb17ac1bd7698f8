"""Measure the per-kernel floor on this box: N dependent trivial kernels, eager vs
hipGraph (torch ops as the trivial kernel), plus a big copy for bandwidth."""
import time
import torch

x = torch.zeros(1, device="cuda")
big = torch.empty(512 * 1024 * 1024 // 4, device="cuda")
big2 = torch.empty_like(big)
N = 2000


def run_eager():
    for _ in range(N):
        x.add_(1.0)


torch.cuda.synchronize()
run_eager()
torch.cuda.synchronize()
t = time.perf_counter()
run_eager()
torch.cuda.synchronize()
eager = (time.perf_counter() - t) / N * 1e6

g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    with torch.cuda.graph(g):
        for _ in range(200):
            x.add_(1.0)
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    g.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t) / 2000 * 1e6

torch.cuda.synchronize()
big2.copy_(big)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    big2.copy_(big)
torch.cuda.synchronize()
bw = 10 * 2 * big.numel() * 4 / (time.perf_counter() - t) / 1e12
print(f"trivial kernel: eager {eager:.2f} us/kernel, graph {graph:.2f} us/kernel; copy bw {bw:.2f} TB/s")
