"""Headline benchmark: output tokens/s + p50 /response latency, Llama-3-8B Q4_K_M
(BASELINE.json metric), measured through the real FastAPI ``/response`` path.

One "step" = one round of ``POST /response`` requests, one per concurrent client
(``--clients``, default 6: K steps post K x C requests), each served exactly as the
reference serves it (reference api.py:118-173): persona system prompt, context
truncation, admission queue, ``create_chat_completion(temperature=1.2,
top_p=0.9, frequency_penalty=0.7, presence_penalty=0.8)`` with no max_tokens -
so each request decodes until EOS or the 1024-token context is full. Whole rounds keep
every client busy to the end of the timed region: a request count that is not a multiple
of C left a last partial wave decoding 1-5 rows alone (round 2's 20 requests at C = 6 spent
~20 % of the timed region on a 2-row tail), which measured the tail, not the serving rate.

GPUs: ``--gpus N`` runs N ranks, one process per GPU. Without ``WORLD_SIZE`` in the
environment and N > 1, bench.py starts ``torch.distributed.run`` itself (before anything
touches a GPU) and exits with its status; under a launcher, ``WORLD_SIZE`` must equal N.

Parallelism (``--parallel``, default ``auto`` = ``dp``; the JSON records both the requested and
the resolved mode):
  * ``tp``: ONE model row-split over the N GPUs (BASELINE configs "8B tensor_split across
    2 MI355X", "70B across 8"): heads / FFN / vocabulary sharded, two all-reduces per
    layer (one-shot P2P kernel over xGMI for decode messages, RCCL for prefill), rank 0
    serves HTTP and drives the continuous batch, ranks 1..N-1 replay its engine commands
    natively. Strong scaling: value = the job's output tokens/s.
  * ``dp``: every GPU an independent replica with its own request stream (the reference's
    deployment model: replicas behind one Service, reference helm/values.yaml:17). Weak
    scaling; value = sum over ranks. The default: a Q4_K_M 8B (5 GB) or 70B (40 GB) fits one
    MI355X's 288 GB many times over, and a decode step sharded N ways pays two all-reduces per
    layer for 1/N of a weight stream that takes ~1.7 ms whole - replicas are the throughput
    configuration; ``tp`` is the latency / memory configuration and stays selectable.

TP pass (``--tp-pass``, default ``auto`` = on when N > 1): after the data-parallel headline is
measured, every rank frees its engine and rank 0 runs ONE tensor-parallel pass over the same N
GPUs in a fresh ``torch.distributed.run`` child (its own process group; the DP ranks wait at a
gloo barrier and touch no GPU meanwhile), bounded by ``--tp-timeout`` seconds. Its result -
tokens/s at C clients, p50, the serial rate, and which comm path each TP message takes with the
rank count RCCL reports (``Engine.comm_info``) - goes into ``config.tp``. The pass's model follows
BASELINE.json's multi-GPU configs (``--tp-model`` default ``auto``): N >= 8 shards Llama-3-70B
Q4_K_M ("70B across 8"), smaller N the headline 8B ("8B tensor_split across 2 MI355X").

Correctness gate of the TP pass (``config.tp.check``): before the child starts, rank 0 records a
TP = 1 reference on its own GPU - the prefill logits of a fixed 48-token prompt and 16 greedy
decode steps with every step's logits (the DP engine when the TP model is the headline model, a
TP = 1 engine of the TP model otherwise: one MI355X holds the 70B). The TP child replays the same
prompt on the sharded engine and compares: every step's logits within ``TP_CHECK_TOL`` of TP = 1
(relative to the largest logit; a wrong shard or a stale peer granule moves them by tens of %),
greedy tokens identical, or diverging only where TP = 1's own logits put the two picks within twice
the deviation measured at that step (a rounding near-tie). A failed check marks the pass failed
(``ok: false``) with the numbers kept. A failed or timed-out pass is recorded in ``config.tp`` with
its error and never touches the DP headline.

Load: ``--clients C`` concurrent clients (default 6 = the reference pod's admission
capacity, 1 in flight + MAX_QUEUE_SIZE 5, reference api.py:19,113) post the K timed
requests; the engine decodes up to ``--max-batch M`` (default = C) of them as rows of one
continuous batch. After the timed run, ``--serial-steps`` requests from ONE client (the
reference's one-generation-at-a-time serving) are timed as well and reported in
``config.serial`` (rank 0's GPU group, same engine).

Admission runs the production settings (the chart's): at most MAX_QUEUE_SIZE + 1 = 6 requests
admitted at once (the reference pod's capacity, reference api.py:19,113), all six decoding as rows
of one batch. Only the server timeout is raised (600 s instead of 25 s, so a slow first request of
a cold box is measured rather than 408'd), and the admission cap only when ``--clients`` exceeds
6; both are recorded in ``bench_overrides``. Weights are random-init of the exact Llama-3-8B Q4_K_M shapes
and type mix (a synthetic GGUF written once per node), prompts are synthetic chat requests.
"""
from __future__ import annotations

import argparse
import asyncio
import datetime
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "output tokens/sec + p50 /response latency, Llama-3-8B Q4_K_M at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # BASELINE.json "published": {} - no reference number exists
BENCH_TIMEOUT_S = 600.0


class CountingEngine:
    """Delegates to the real engine and records usage per /response."""
    supports_cancel = True

    def __init__(self, llm):
        self.llm = llm
        self.completion_tokens = []
        self.prompt_tokens = []
        self.decode_s = []

    @property
    def batch_width(self):
        return self.llm.batch_width

    def n_ctx(self):
        return self.llm.n_ctx()

    def create_chat_completion(self, **kw):
        out = self.llm.create_chat_completion(**kw)
        self.completion_tokens.append(out["usage"]["completion_tokens"])
        self.prompt_tokens.append(out["usage"]["prompt_tokens"])
        self.decode_s.append(out["timings"]["decode_s"])
        return out

    def health(self):
        return self.llm.health()


def _sched_stats(eng) -> dict:
    """The batch scheduler's counters (admitted, joint / chunked admissions), if the backend has one."""
    try:
        h = eng.health()
    except Exception:
        return {}
    b = h.get("batching") if isinstance(h, dict) else None
    return dict(b) if isinstance(b, dict) else {}


def make_request(i: int) -> dict:
    names = ["Mia.f", "Leo", "Ava.f", "Max"]
    ctx = []
    for j in range(6):
        turn = "user" if j % 2 == 0 else "assistant"
        ctx.append({"turn": turn, "message": f"message {i}-{j}: tell me something fun about the number {i * 7 + j} "
                                              "and how you would spend a rainy afternoon in a small seaside town."})
    return {"bot_profile": {"name": names[i % 4], "appearance": "tall, brown hair, green eyes, freckles, smiles"},
            "user_profile": {"name": "bench"}, "context": ctx}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# torchrun's per-rank environment: a TP-pass child must start a launcher of its own without it
_LAUNCHER_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                  "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def resolve_tp_model(args, world: int) -> str:
    """The TP pass's model: BASELINE.json's multi-GPU configs - "70B across 8" at N >= 8, the
    headline 8B ("8B tensor_split across 2") below; an explicit --tp-model wins."""
    if args.tp_model and args.tp_model != "auto":
        return args.tp_model
    return "llama3-70b-q4_k_m" if world >= 8 else args.model


def tp_pass_cmd(args, world: int, json_out: str, check_ref: str = "") -> list:
    """The TP child: this script under its own torch.distributed.run, --parallel tp over `world` GPUs."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
           "--gpus", str(world), "--parallel", "tp", "--model", resolve_tp_model(args, world),
           "--steps", str(args.tp_steps), "--warmup", "1", "--serial-steps", "1", "--tp-pass", "off",
           "--clients", str(args.clients), "--max-batch", str(args.max_batch), "--n-ctx", str(args.n_ctx),
           "--model-dir", args.model_dir, "--json-out", json_out]
    if check_ref:
        cmd += ["--tp-check-ref", check_ref]
    return cmd


# ------------------------------------------------------------------ TP correctness gate
TP_CHECK_PROMPT = 48      # prompt tokens (one prefill chunk)
TP_CHECK_STEPS = 16       # greedy decode steps
TP_CHECK_TOL = 0.15       # per-step logits vs TP = 1: max |difference| relative to the largest |logit|
TP_CHECK_COS = 0.99       # ... and cosine similarity of the logit vectors
# (rounding noise measured on the one-GPU TP = 2 rehearsal, 8B, 32 layers: max relative deviation
# 0.35 % at the prefill and up to 2.7 % on the decode steps, which read the K / V the prefill's
# f16 roundings wrote; deeper models accumulate more. A wrong shard or a stale granule gives
# unrelated logits: cosine far below 0.99)


def _rel(a, b) -> float:
    import numpy as np
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def tp_check_prompt(n_vocab: int) -> list:
    import numpy as np
    return [int(t) for t in np.random.default_rng(2024).integers(3, min(n_vocab, 30000), TP_CHECK_PROMPT)]


def tp_check_record(eng, n_vocab: int, steps: int = TP_CHECK_STEPS):
    """Greedy run of the fixed prompt on an engine (eval_logits / decode_logits on slot 0):
    (tokens, logits per step [steps + 1, V]) - row 0 is the prefill's."""
    import numpy as np
    prompt = tp_check_prompt(n_vocab)
    rows = [np.asarray(eng.eval_logits(prompt, 0), np.float32)[:n_vocab]]
    toks = []
    for k in range(steps):
        t = int(np.argmax(rows[-1]))
        toks.append(t)
        rows.append(np.asarray(eng.decode_logits(t, len(prompt) + k), np.float32)[:n_vocab])
    return np.asarray(toks, np.int64), np.stack(rows)


def _cos(a, b) -> float:
    import numpy as np
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.dot(a, b) / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-30))


def tp_check_compare(ref_toks, ref_logits, toks, logits, tol: float = TP_CHECK_TOL,
                     cos_min: float = TP_CHECK_COS) -> dict:
    """The gate: logits of every step both runs fed identically within `tol` of TP = 1 and at
    cosine >= `cos_min`; greedy tokens equal, or diverging where TP = 1's logits of the two picks
    lie within twice the deviation measured at that step."""
    import numpy as np
    n = min(len(ref_toks), len(toks))
    dev, cos, div, gap = [], [], None, None
    for k in range(n + 1):
        if k < len(ref_logits) and k < len(logits):
            dev.append(_rel(logits[k], ref_logits[k]))
            cos.append(_cos(logits[k], ref_logits[k]))
        if k == n:
            break
        if int(toks[k]) != int(ref_toks[k]):
            div = k
            r = np.asarray(ref_logits[k], np.float64)
            gap = float(abs(r[int(toks[k])] - r[int(ref_toks[k])]) / max(np.abs(r).max(), 1e-12))
            break
    ok_logits = bool(dev) and max(dev) <= tol and min(cos) >= cos_min
    ok_greedy = len(toks) == len(ref_toks) and (div is None or gap <= 2.0 * dev[div])
    return {"status": "passed" if ok_logits and ok_greedy else "failed",
            "prompt_tokens": TP_CHECK_PROMPT, "greedy_steps": int(len(ref_toks)),
            "max_rel_dev_vs_tp1": round(max(dev), 6) if dev else None,
            "prefill_rel_dev_vs_tp1": round(dev[0], 6) if dev else None, "tol": tol,
            "min_cosine_vs_tp1": round(min(cos), 6) if cos else None, "cos_min": cos_min,
            "greedy_identical_steps": int(div if div is not None else n),
            "divergence": None if div is None else {"step": div, "tp1_gap": round(gap, 6),
                                                     "allowed": round(2.0 * dev[div], 6)}}


def tp_check_save(path: str, toks, logits):
    import numpy as np
    np.savez(path, toks=np.asarray(toks, np.int64), logits=np.asarray(logits, np.float32))


def tp_check_load(path: str):
    import numpy as np
    with np.load(path) as z:   # (allow_pickle stays False: plain arrays written by tp_check_save)
        return z["toks"], z["logits"]


def run_tp_pass(cmd: list, json_out: str, timeout_s: float, heartbeat_s: float = 60.0) -> dict:
    """Run the TP child (its own session, launcher variables dropped) for at most `timeout_s`;
    returns its result block, or {"ok": False, "error": ...} - it never raises."""
    t0 = time.time()
    log_path = json_out + ".log"
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCHER_VARS and not k.startswith("TORCHELASTIC_")}
    try:
        with open(log_path, "w") as log:
            proc = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
            next_beat = t0 + heartbeat_s
            while proc.poll() is None:
                now = time.time()
                if now - t0 > timeout_s:
                    try:
                        os.killpg(proc.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    proc.wait()
                    raise TimeoutError(f"TP pass timed out after {timeout_s:.0f} s")
                if now >= next_beat:
                    print(f"[bench] tp pass running ({now - t0:.0f} s)", file=sys.stderr, flush=True)
                    next_beat += heartbeat_s
                time.sleep(0.5)
        if proc.returncode != 0:
            raise RuntimeError(f"TP pass exited with status {proc.returncode}")
        with open(json_out) as f:
            res = json.load(f)
    except Exception as e:
        tail = ""
        try:
            with open(log_path, errors="replace") as f:
                text = f.read()
            # the ranks' own errors first (torchrun's summary traceback fills the tail)
            errs = [l for l in text.splitlines() if ("Error" in l or "error" in l or "Exception" in l)
                    and "torch/distributed" not in l and "elastic" not in l][:12]
            tail = "\n".join(errs) + "\n...\n" + text[-1500:]
        except OSError:
            pass
        return {"ok": False, "error": f"{type(e).__name__}: {e}", "wall_s": round(time.time() - t0, 1),
                "log": log_path, "log_tail": tail}
    cfg = res.get("config", {})
    check = cfg.get("check")
    out = {"ok": True, "model": cfg.get("model"), "parallelism": cfg.get("parallelism"), "scaling": "strong",
           "value": res.get("value"), "unit": res.get("unit"), "ms_per_step": res.get("ms_per_step"),
           "p50_response_ms": cfg.get("p50_response_ms"), "requests": cfg.get("requests"),
           "avg_output_tokens": cfg.get("avg_output_tokens"), "serial": cfg.get("serial"),
           "comm": cfg.get("comm"), "check": check, "wall_s": round(time.time() - t0, 1)}
    if check is not None and check.get("status") != "passed":
        # a fast number from a wrong model is no result: the pass fails, its numbers are kept
        out["ok"] = False
        out["error"] = "TP correctness check failed against the TP = 1 reference"
    return out


def tp_reference_engine(args, tp_model: str, device: int, ref_path: str):
    """The TP = 1 reference of a TP model other than the headline one (the 70B at N >= 8): its
    synthetic GGUF (written once; the TP child reuses it) on ONE GPU, the fixed greedy run recorded,
    the engine freed before the child starts. -> (ref_path, None) or ("", error)."""
    try:
        from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
        from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
        path = os.path.join(args.model_dir, f"{tp_model}-s0.gguf")
        if not os.path.exists(path):
            t0 = time.time()
            write_synthetic_gguf(tp_model, path, seed=0)
            print(f"[bench] wrote synthetic {tp_model} in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        ref = Llama(path, n_gpu_layers=-1, n_ctx=args.n_ctx, split_mode="none", verbose=False, device=device)
        try:
            tp_check_save(ref_path, *tp_check_record(ref._backend.engine, ref.n_vocab()))
        finally:
            ref.close()
            del ref
            import gc
            gc.collect()
        return ref_path, None
    except Exception as e:
        return "", f"{type(e).__name__}: {e}"


def _launch_ranks(n: int) -> int:
    """Start n ranks of this script under torch.distributed.run (no GPU touched here)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b-q4_k_m")
    ap.add_argument("--parallel", choices=["auto", "dp", "tp"], default="auto")
    ap.add_argument("--n-ctx", type=int, default=1024)
    ap.add_argument("--clients", type=int, default=6, help="concurrent clients posting /response")
    ap.add_argument("--max-batch", type=int, default=0, help="continuous-batch rows (0 = --clients)")
    ap.add_argument("--serial-steps", type=int, default=-1,
                    help="requests of the one-client serial run after the timed run (-1: max(2, steps // 4))")
    ap.add_argument("--model-dir", default=os.environ.get("SYNTH_MODEL_DIR", os.path.join(
        os.environ.get("TMPDIR", "/tmp"), "llama_amd_models")))
    ap.add_argument("--tp-pass", choices=["auto", "on", "off"], default="auto",
                    help="N > 1: a tensor-parallel pass over the same GPUs after the DP headline (config.tp)")
    ap.add_argument("--tp-model", default="auto",
                    help="model of the TP pass (auto: llama3-70b-q4_k_m at N >= 8, else --model)")
    ap.add_argument("--tp-check-ref", default="",
                    help="(TP child) TP = 1 reference (.npz) to check the sharded engine against")
    ap.add_argument("--tp-steps", type=int, default=2, help="timed rounds of the TP pass")
    ap.add_argument("--tp-timeout", type=float, default=480.0, help="wall bound of the TP pass (s)")
    ap.add_argument("--json-out", default="", help="also write rank 0's JSON result to this file")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return _launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    parallel = args.parallel if args.parallel != "auto" else "dp"
    # Rehearsal mode: LFK_BENCH_DEVICE=<d> puts every rank on GPU d (a one-GPU box running the
    # N-rank flow); RCCL refuses two ranks on one device, so TP collectives take the P2P kernel
    # for every message (comm=ipc) and the bench's own reductions go over gloo.
    rehearse = os.environ.get("LFK_BENCH_DEVICE")
    device = int(rehearse) if rehearse is not None else local

    import torch
    import torch.distributed as dist
    tp_pass = world > 1 and parallel == "dp" and args.tp_pass != "off"
    if world > 1:
        # control plane only (barriers, object broadcasts): the engine runs its own collectives.
        # (the DP ranks wait out rank 0's TP pass at a barrier: the timeout covers it)
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=1800 + args.tp_timeout))

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)

    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    os.makedirs(args.model_dir, exist_ok=True)
    path = os.path.join(args.model_dir, f"{args.model}-s0.gguf")
    if (rank if rehearse is not None else local) == 0 and not os.path.exists(path):
        t0 = time.time()
        write_synthetic_gguf(args.model, path, seed=0)
        print(f"[bench] wrote synthetic {args.model} in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()

    from llama_fastapi_k8s_gpu_amd.config import Settings
    from llama_fastapi_k8s_gpu_amd.engine.llama import Llama
    from llama_fastapi_k8s_gpu_amd.server.app import create_app

    t0 = time.time()
    tp = parallel == "tp" and world > 1
    max_batch = args.max_batch or args.clients
    extra = {"max_batch": max_batch} if max_batch > 1 else {}
    if tp:
        extra.update(tp_comm="ipc" if rehearse is not None else "auto", device=device)
    elif rehearse is not None:
        extra.update(device=device)
    llm = Llama(path, n_gpu_layers=-1, n_ctx=args.n_ctx, seed=1234 + (0 if tp else rank),
                split_mode="row" if tp else "none", verbose=False, **extra)
    print(f"[bench] rank {rank}: loaded in {time.time() - t0:.1f}s ({llm.backend_name}, parallel={parallel})",
          file=sys.stderr, flush=True)
    if tp and rank > 0:
        # follower: replay rank 0's engine commands until it closes the group
        llm.follow()
        llm.close()
        dist.barrier()
        dist.destroy_process_group()
        return 0

    comm = llm._backend.engine.comm_info() if tp and hasattr(getattr(llm, "_backend", None), "engine") else None
    check = None
    if tp and args.tp_check_ref:
        # the correctness gate: the fixed prompt's greedy run on the sharded engine against TP = 1
        try:
            ref_toks, ref_logits = tp_check_load(args.tp_check_ref)
            got_toks, got_logits = tp_check_record(llm._backend.engine, llm.n_vocab(), len(ref_toks))
            check = tp_check_compare(ref_toks, ref_logits, got_toks, got_logits)
        except Exception as e:
            check = {"status": "failed", "error": f"{type(e).__name__}: {e}"}
        print(f"[bench] tp check: {check}", file=sys.stderr, flush=True)
    eng = CountingEngine(llm)
    settings = Settings()
    settings.timeout_seconds = BENCH_TIMEOUT_S  # measure latency, do not 408 long generations in the bench
    settings.max_batch = max_batch
    # production admission (MAX_QUEUE_SIZE + 1 = 6 admitted at once); raised only for more clients
    if args.clients > settings.admission_cap:
        settings.max_admitted = args.clients
    app = create_app(settings, engine=eng)
    serial_steps = args.serial_steps if args.serial_steps >= 0 else max(2, args.steps // 4)

    import httpx

    latencies, serial_lat = [], []

    async def run():
        async with app.router.lifespan_context(app):
            transport = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=transport, base_url="http://bench", timeout=BENCH_TIMEOUT_S) as c:
                async def drive(ids, lat, clients):
                    todo = list(ids)

                    async def client():
                        while todo:
                            i = todo.pop(0)
                            t = time.perf_counter()
                            r = await c.post("/response", json=make_request(i))
                            assert r.status_code == 200, r.text
                            if lat is not None:
                                lat.append(time.perf_counter() - t)
                    await asyncio.gather(*[client() for _ in range(max(1, clients))])
                nc = max(1, args.clients)
                await drive(range(1000, 1000 + args.warmup * nc), None, args.clients)
                if not tp:
                    barrier()
                else:
                    torch.cuda.synchronize(device)
                n0 = len(eng.completion_tokens)
                st0 = _sched_stats(eng)
                t_start = time.perf_counter()
                await drive(range(args.steps * nc), latencies, args.clients)
                # TP: rank 0's last step completed its all-reduces, so every rank is done with it
                if not tp:
                    barrier()
                else:
                    torch.cuda.synchronize(device)
                elapsed = time.perf_counter() - t_start
                n1 = len(eng.completion_tokens)
                st1 = _sched_stats(eng)
                ts = time.perf_counter()
                if serial_steps > 0:
                    await drive(range(2000, 2000 + serial_steps), serial_lat, 1)
                # the continuous batch's admissions over the timed rounds (how the C requests of a
                # round entered: one joint prefill, or several)
                sched = ({k: st1[k] - st0.get(k, 0) for k in ("admitted", "joint_admissions", "chunked_admissions")
                          if isinstance(st1.get(k), (int, float))} if st1 else None)
                return elapsed, n0, n1, time.perf_counter() - ts, sched

    elapsed, n0, n1, serial_s, sched = asyncio.run(run())
    llm.close()   # TP: publishes STOP, the followers' follow() returns
    del app, eng.llm
    toks = sum(eng.completion_tokens[n0:n1])
    ptoks = sum(eng.prompt_tokens[n0:n1])
    s_toks = sum(eng.completion_tokens[n1:])
    if world > 1 and not tp:
        dev = "cpu"
        t = torch.tensor([elapsed, float(toks)], dtype=torch.float64, device=dev)
        tmax = t[0].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, total = float(tmax), float(t[1])
    else:
        total = float(toks)
    value = total / elapsed
    p50 = statistics.median(latencies) * 1e3
    dec = sum(eng.decode_s[n0:n1])
    if rank == 0:
        # the model this run served (the headline config is the default llama3-8b-q4_k_m)
        from llama_fastapi_k8s_gpu_amd.gguf.synthetic import SPECS
        _spec = SPECS.get(args.model)
        model_label = ("Llama-3-8B Q4_K_M" if args.model == "llama3-8b-q4_k_m"
                       else f"{_spec.name} {_spec.quant.upper()}" if _spec is not None else args.model)
        res = {
            # BASELINE.json's metric string names the headline model; another --model names itself
            "metric": METRIC if args.model == "llama3-8b-q4_k_m" else METRIC.replace("Llama-3-8B Q4_K_M", model_label),
            "value": round(value, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "strong" if tp else "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "q4_k_m weights; f16 (batched decode and prompt prefill MFMA, tile16 copies) / int8 "
                     "(single-row GEMV) activations; fp32 accumulate",
            "data": f"synthetic (random-init {model_label} GGUF, synthetic chat requests)",
            "config": {"model": model_label,
                       "global_batch": (1 if tp else world) * min(args.clients, max_batch),
                       "seq_len": args.n_ctx, "parallelism": f"{'tp' if tp else 'dp'}{world}",
                       "parallel_requested": args.parallel,
                       "clients_per_group": args.clients, "max_batch": max_batch,
                       "p50_response_ms": round(p50, 1),
                       "decode_tokens_per_s_per_request": round(toks / dec, 1) if dec > 0 else None,
                       "requests": n1 - n0, "step": f"one round of {args.clients} concurrent /response requests",
                       "avg_prompt_tokens": round(ptoks / max(1, n1 - n0), 1),
                       "avg_output_tokens": round(toks / max(1, n1 - n0), 1),
                       "serial": {"requests": serial_steps, "clients": 1,
                                  "tokens_per_s": round(s_toks / serial_s, 2) if serial_steps else None,
                                  "p50_response_ms": round(statistics.median(serial_lat) * 1e3, 1)
                                  if serial_lat else None,
                                  "scope": "rank 0's GPU group" if world > 1 else "whole job"},
                       "admission": {"max_queue_size": settings.max_queue_size,
                                     "admission_cap": settings.admission_cap, "max_batch": max_batch},
                       "bench_overrides": {"timeout_seconds": BENCH_TIMEOUT_S,
                                           **({"admission_cap": settings.admission_cap}
                                              if settings.max_admitted is not None else {}),
                                           "production": {"timeout_seconds": 25.0, "max_queue_size": 5,
                                                          "admission_cap": 6}}},
        }
        if sched:
            res["config"]["scheduler"] = sched
        if comm is not None:
            res["config"]["comm"] = comm
        if check is not None:
            res["config"]["check"] = check
    # the TP pass's TP = 1 reference (rank 0, its own GPU): the DP engine when the TP model is the
    # headline model, recorded before that engine goes
    tp_model = resolve_tp_model(args, world) if tp_pass else ""
    ref_path, ref_err = "", None
    if tp_pass and rank == 0:
        ref_path = os.path.join(tempfile.gettempdir(), f"lfk_bench_tpref_{os.getpid()}.npz")
        if tp_model == args.model:
            try:
                tp_check_save(ref_path, *tp_check_record(llm._backend.engine, llm.n_vocab()))
            except Exception as e:
                ref_path, ref_err = "", f"{type(e).__name__}: {e}"
    # the TP pass: every rank's engine is gone (its memory with it); rank 0 runs the child while
    # the others wait at the barrier below
    del llm
    import gc
    gc.collect()
    if tp_pass:
        dist.barrier()
        if rank == 0:
            if tp_model != args.model and ref_path:
                ref_path, ref_err = tp_reference_engine(args, tp_model, device, ref_path)
            print(f"[bench] tp pass: tp{world} over {tp_model}", file=sys.stderr, flush=True)
            out = os.path.join(tempfile.gettempdir(), f"lfk_bench_tp{world}_{os.getpid()}.json")
            tpres = run_tp_pass(tp_pass_cmd(args, world, out, ref_path), out, args.tp_timeout)
            if not ref_path and tpres.get("ok"):
                # no TP = 1 reference: the pass's number is unverified, so it does not count
                tpres.update(ok=False, check={"status": "failed", "error": f"no TP = 1 reference: {ref_err}"},
                             error="TP correctness check unavailable")
            res["config"]["tp"] = tpres
    if rank == 0:
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(res, f)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
