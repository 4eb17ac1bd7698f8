"""P2P all-reduce / all-gather latency (kernels/p2p_allreduce.hip) at 2 / 4 / 8 ranks.

    python tools/p2p_latency.py --ranks 2,4,8 [--json out.json]

Every rank is a process on device 0 (the one-GPU box's rehearsal of the one-process-per-GPU
layout, `comm="ipc"`): regions exported with hipIpc handles, exchanged over gloo, opened, then
per message size a hipGraph of `--reps` back-to-back collectives is replayed after a barrier and
timed with events on every rank (the max over ranks is reported, us per collective). The sizes
are the decode step's messages: one 8B row (4096 floats), one 70B row (8192), six rows of each
(the B = 6 batch step). On one device the peers' stores and flag polls stay in one L2/MALL, so
this is the kernel's own latency chain (launch, push, flag hand-off, rank-order sum) without the
xGMI hop; an 8-GPU node adds the link latency (~1-2 us per hop) on top.
"""
import argparse
import json
import os
import sys

SIZES = [4096, 8192, 6 * 4096, 6 * 8192]


def _worker(rank, world, port, reps, q, stress=0):
    try:
        # one hardware queue per process: 8 processes x the default 4 queues oversubscribe the
        # scheduler, which then time-slices the queues (~10 ms per collective measured, r4)
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        from llama_fastapi_k8s_gpu_amd.parallel.comm import allgather_bytes
        from llama_fastapi_k8s_gpu_amd.runtime import load_hip
        hip = load_hip()
        c = hip.P2PComm(rank, world, max(SIZES), 0)
        c.open(allgather_bytes(c.handle()))
        out = {}
        if stress:
            # mixed sizes back to back, eager, no host barrier between launches: checked sums
            s = torch.cuda.current_stream().cuda_stream
            bad = 0
            for it in range(stress):
                n = [SIZES[-1], 37, 1000 + it % 97, 4096][it % 4]
                x = torch.full((n,), float(rank + 1), device="cuda")
                y = torch.empty(n * (world if it % 5 == 0 else 1), device="cuda")
                (c.allgather if it % 5 == 0 else c.allreduce)(x.data_ptr(), y.data_ptr(), n, s)
                if it % 25 == 0:
                    torch.cuda.synchronize()
                    want = float(world * (world + 1) // 2)
                    bad += int(it % 5 != 0 and not bool((y == want).all()))
            torch.cuda.synchronize()
            out["stress_bad"] = bad
            q.put((rank, out, c.error(), None))
            dist.barrier()
            dist.destroy_process_group()
            return
        for op in ("allreduce", "allgather"):
            for n in SIZES:
                src = torch.randn(n, device="cuda")
                dst = torch.empty(n * (world if op == "allgather" else 1), device="cuda")
                fn = getattr(c, op)
                cs = torch.cuda.Stream()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(cs):
                    fn(src.data_ptr(), dst.data_ptr(), n, cs.cuda_stream)   # warm (outside the graph)
                    with torch.cuda.graph(g, stream=cs):
                        for _ in range(reps):
                            fn(src.data_ptr(), dst.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                times = []
                for _ in range(3):
                    dist.barrier()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    times.append(e0.elapsed_time(e1) * 1e3 / reps)
                out[f"{op}_{n}"] = min(times)
        q.put((rank, out, c.error(), None))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put((rank, None, -1, traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default="")
    ap.add_argument("--stress", type=int, default=0, help="instead: this many mixed-size eager collectives, checked")
    args = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    res = {"what": "P2P collective latency, us per op (max over ranks), all ranks on device 0 (IPC mode)",
           "sizes_floats": SIZES, "reps": args.reps}
    for i, world in enumerate(int(r) for r in args.ranks.split(",")):
        q = ctx.Queue()
        port = 29800 + (os.getpid() % 500) + 11 * i
        procs = [ctx.Process(target=_worker, args=(r, world, port, args.reps, q, args.stress)) for r in range(world)]
        for p in procs:
            p.start()
        got = [q.get(timeout=300) for _ in procs]
        for p in procs:
            p.join(timeout=60)
        errs = [g[3] for g in got if g[3]]
        if errs:
            raise SystemExit(errs[0])
        if any(g[2] for g in got):
            raise SystemExit(f"device error words: {[g[2] for g in got]}")
        res[f"world{world}"] = {k: round(max(g[1][k] for g in got), 2) for k in got[0][1]}
        print(world, res[f"world{world}"], flush=True)
    print(json.dumps(res))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
