"""bench.py's tensor-parallel pass orchestration on the CPU (the GPU run is the driver's
multi-GPU bench): the child command, result capture, and failures recorded - never raised - so a
broken TP pass cannot zero the data-parallel headline."""
import argparse
import json
import sys
import time

import bench


def _args(**kw):
    a = dict(tp_model="", model="llama3-8b-q4_k_m", tp_steps=2, clients=6, max_batch=0, n_ctx=1024,
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
