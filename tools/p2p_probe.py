"""Host-only probe of the P2P receive-region IPC mappings (no kernel launch, no peer access):
two ranks on device 0 create their regions, optionally free and re-allocate device memory
(--junk: before the handle export, as the engine's setup can), exchange handles, open them,
and print every mapping's (pointer, allocation base, allocation size) and the raw handle bytes.

    python tools/p2p_probe.py [--junk] [--uncached]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, junk, uncached, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from llama_fastapi_k8s_gpu_amd.parallel.comm import allgather_bytes
        from llama_fastapi_k8s_gpu_amd.runtime import load_hip
        hip = load_hip()
        pre = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")   # something allocated before
        c = hip.P2PComm(rank, world, 4096, 0, uncached=uncached)
        own0 = c.mappings()[rank]
        if junk:
            j = [torch.empty(3 << 20, dtype=torch.uint8, device="cuda") for _ in range(4)]
            del j
            torch.cuda.empty_cache()
            keep = torch.full((5 << 20,), 7, dtype=torch.uint8, device="cuda")  # noqa: F841
        h = c.handle()
        hs = allgather_bytes(h)
        c.open(hs)
        q.put((rank, {"own_at_create": [hex(v) for v in own0], "mappings": [[hex(v) for v in m] for m in c.mappings()],
                      "handle": h.hex(), "pre": hex(pre.data_ptr())}, None))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put((rank, None, traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--junk", action="store_true")
    ap.add_argument("--uncached", action="store_true")
    args = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=worker, args=(r, 2, port, args.junk, args.uncached, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        r, info, err = q.get(timeout=120)
        out[r] = info if err is None else err
    for p in ps:
        p.join(30)
    print(json.dumps({"junk": args.junk, "uncached": args.uncached, "ranks": out}, indent=1))


if __name__ == "__main__":
    main()
