"""bench.py's tensor-parallel pass orchestration on the CPU (the GPU run is the driver's
multi-GPU bench): the child command, result capture, and failures recorded - never raised - so a
broken TP pass cannot zero the data-parallel headline."""
import argparse
import json
import sys
import time

import bench


def _args(**kw):
    a = dict(tp_model="auto", model="llama3-8b-q4_k_m", tp_steps=2, clients=6, max_batch=0, n_ctx=1024,
             model_dir="/tmp/m", tp_timeout=480.0)
    a.update(kw)
    return argparse.Namespace(**a)


def test_tp_pass_command_is_a_fresh_tp_launch():
    cmd = bench.tp_pass_cmd(_args(tp_model="llama3-70b-q4_k_m"), 8, "/tmp/out.json")
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    i = cmd.index("--parallel")
    assert cmd[i + 1] == "tp"
    assert cmd[cmd.index("--tp-pass") + 1] == "off"           # the child runs no pass of its own
    assert cmd[cmd.index("--model") + 1] == "llama3-70b-q4_k_m"
    assert cmd[cmd.index("--gpus") + 1] == "8" and cmd[cmd.index("--json-out") + 1] == "/tmp/out.json"
    assert bench.tp_pass_cmd(_args(), 2, "/x")[bench.tp_pass_cmd(_args(), 2, "/x").index("--model") + 1] == \
        "llama3-8b-q4_k_m"


def test_tp_pass_result_and_clean_launcher_env(tmp_path, monkeypatch):
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("MASTER_PORT", "1234")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "x")
    out = str(tmp_path / "r.json")
    child = ("import json, os, sys\n"
             "res = {'value': 123.4, 'unit': 'tokens/s', 'ms_per_step': 10.0,\n"
             "       'config': {'model': 'M', 'parallelism': 'tp2', 'p50_response_ms': 5.0, 'requests': 12,\n"
             "                  'serial': {'tokens_per_s': 50.0},\n"
             "                  'comm': {'rccl_comm_ranks': '2', 'env_rank': os.environ.get('RANK'),\n"
             "                           'env_ws': os.environ.get('WORLD_SIZE'),\n"
             "                           'elastic': os.environ.get('TORCHELASTIC_RUN_ID')}}}\n"
             "json.dump(res, open(sys.argv[1], 'w'))\n")
    r = bench.run_tp_pass([sys.executable, "-c", child, out], out, timeout_s=60)
    assert r["ok"] and r["value"] == 123.4 and r["parallelism"] == "tp2" and r["scaling"] == "strong"
    assert r["p50_response_ms"] == 5.0 and r["serial"] == {"tokens_per_s": 50.0}
    # the child started with no torchrun variables of the parent's rank
    assert r["comm"]["rccl_comm_ranks"] == "2"
    assert r["comm"]["env_rank"] is None and r["comm"]["env_ws"] is None and r["comm"]["elastic"] is None


def test_tp_pass_failure_is_recorded(tmp_path):
    out = str(tmp_path / "r.json")
    r = bench.run_tp_pass([sys.executable, "-c", "print('rank 1: boom'); raise SystemExit(3)"], out, timeout_s=60)
    assert r["ok"] is False and "status 3" in r["error"] and "boom" in r["log_tail"]
    json.dumps(r)   # serialisable into the bench line


def test_tp_pass_timeout_kills_the_child(tmp_path):
    out = str(tmp_path / "r.json")
    t0 = time.time()
    r = bench.run_tp_pass([sys.executable, "-c", "import time; time.sleep(60)"], out, timeout_s=1.5,
                          heartbeat_s=0.5)
    assert r["ok"] is False and "timed out" in r["error"]
    assert time.time() - t0 < 20


def test_tp_model_follows_the_baseline_configs():
    """--tp-model auto: "70B across 8" at N >= 8, the headline 8B ("8B across 2") below; an explicit
    model wins. The child command carries the resolved model and the reference path."""
    assert bench.resolve_tp_model(_args(), 8) == "llama3-70b-q4_k_m"
    assert bench.resolve_tp_model(_args(), 2) == "llama3-8b-q4_k_m"
    assert bench.resolve_tp_model(_args(), 4) == "llama3-8b-q4_k_m"
    assert bench.resolve_tp_model(_args(tp_model="tiny-llama3-tp"), 8) == "tiny-llama3-tp"
    cmd = bench.tp_pass_cmd(_args(), 8, "/o.json", "/ref.npz")
    assert cmd[cmd.index("--model") + 1] == "llama3-70b-q4_k_m"
    assert cmd[cmd.index("--tp-check-ref") + 1] == "/ref.npz"
    assert "--tp-check-ref" not in bench.tp_pass_cmd(_args(), 2, "/o.json")


class _FakeEngine:
    """eval_logits / decode_logits of a deterministic toy model (the next token's logits depend on
    the last token and the position); `bias` perturbs it like a TP engine's rounding or a bad shard."""

    def __init__(self, V=97, bias=None):
        import numpy as np
        self.V, self.bias = V, bias
        self.W = np.random.default_rng(0).standard_normal((V, V)).astype(np.float32)

    def _row(self, tok, pos):
        import numpy as np
        r = self.W[tok % self.V] * (1.0 + 0.01 * pos)
        return r + (self.bias(tok, pos) if self.bias else 0.0)

    def eval_logits(self, toks, pos):
        return self._row(toks[-1], pos + len(toks) - 1)

    def decode_logits(self, tok, pos):
        return self._row(tok, pos)


def test_tp_check_gate(tmp_path):
    import numpy as np
    ref = _FakeEngine()
    rt, rl = bench.tp_check_record(ref, ref.V)
    assert rl.shape == (bench.TP_CHECK_STEPS + 1, ref.V) and len(rt) == bench.TP_CHECK_STEPS
    # the recorded reference round-trips through the .npz the child loads
    bench.tp_check_save(str(tmp_path / "ref.npz"), rt, rl)
    lt, ll = bench.tp_check_load(str(tmp_path / "ref.npz"))
    assert (lt == rt).all() and np.allclose(ll, rl)
    # identical engine: passed, no divergence
    c = bench.tp_check_compare(lt, ll, *bench.tp_check_record(_FakeEngine(), ref.V))
    assert c["status"] == "passed" and c["divergence"] is None and c["max_rel_dev_vs_tp1"] == 0.0
    # rounding-sized noise: passed
    noisy = _FakeEngine(bias=lambda t, p: 1e-4 * np.sin(np.arange(97) * (t + 1)))
    assert bench.tp_check_compare(rt, rl, *bench.tp_check_record(noisy, ref.V))["status"] == "passed"
    # a wrong shard (logits off by tens of %): failed
    bad = _FakeEngine(bias=lambda t, p: 0.8 * np.cos(np.arange(97) * 0.37 * (t + 2)))
    c = bench.tp_check_compare(rt, rl, *bench.tp_check_record(bad, ref.V))
    assert c["status"] == "failed" and c["min_cosine_vs_tp1"] < bench.TP_CHECK_COS


def test_tp_check_greedy_divergence_rule():
    """A greedy divergence passes only at a near-tie of TP = 1's own logits (gap within twice the
    deviation measured at that step)."""
    import numpy as np
    V, n = 8, 4
    ref_logits = np.zeros((n + 1, V), np.float32)
    ref_logits[:, 0] = 10.0
    ref_logits[2, 1] = 9.99          # step 2: token 1 is a near-tie of token 0
    ref_toks = np.zeros(n, np.int64)
    got_logits = ref_logits.copy()
    got_logits[2, 1] = 10.01         # TP's rounding flips the pick at step 2 (dev 1e-3 at that step)
    got_toks = np.array([0, 0, 1, 0])
    c = bench.tp_check_compare(ref_toks, ref_logits, got_toks, got_logits)
    assert c["status"] == "passed" and c["divergence"]["step"] == 2
    # the same divergence where TP = 1 had a clear winner: failed
    ref_logits[2, 1] = 5.0
    got_logits[2, 1] = 10.5
    c = bench.tp_check_compare(ref_toks, ref_logits, got_toks, got_logits)
    assert c["status"] == "failed"


def test_failed_check_marks_the_pass_failed(tmp_path):
    out = str(tmp_path / "r.json")
    child = ("import json, sys\n"
             "json.dump({'value': 99.0, 'config': {'check': {'status': 'failed', 'max_rel_dev_vs_tp1': 0.4}}},"
             " open(sys.argv[1], 'w'))\n")
    r = bench.run_tp_pass([sys.executable, "-c", child, out], out, timeout_s=60)
    assert r["ok"] is False and "correctness" in r["error"] and r["value"] == 99.0
    assert r["check"]["status"] == "failed"
