"""A follower's failure reaches rank 0 (reference api.py:76-78,171-173 turn engine
errors into 500): the 2-rank tensor-parallel server of tests/test_serve_tp_gpu.py, with the test
hook LFK_TP_FAULT making rank 1 fail its 4th engine command - as a host failure (published over
the control channel) or as a device-side fault word (what a timed-out collective wait stores into
every rank's region). Either way the request in flight gets 500, /health turns 503 with the
failing rank named, and the poisoned group refuses further requests instead of serving answers
computed from a diverged rank."""
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.error
import urllib.request

import pytest

pytestmark = pytest.mark.gpu

BODY = {"bot_profile": {"name": "Mia.f", "appearance": "a, b, c, d"}, "user_profile": {"name": "u"},
        "context": [{"turn": "user", "message": "hello there, tell me a long story"}]}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _get(url, timeout=5.0):
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def _post(url, timeout=120.0):
    req = urllib.request.Request(url, data=json.dumps(BODY).encode(), headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind", ["host", "dev"])
def test_follower_fault_fails_requests_and_health(tmp_path, kind):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    path = write_synthetic_gguf("tiny-llama3-tp", str(tmp_path / "tp.gguf"), seed=4)
    port, mport = _free_port(), _free_port()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MODEL_PATH=path, SPLIT_MODE="row", TP_COMM="ipc", TP_DEVICE="0", HOST="127.0.0.1",
               PORT=str(port), N_CTX="256", N_BATCH="64", MAX_BATCH="3", SEED="5", PYTHONPATH=root,
               LFK_TP_FAULT="1:4" + (":dev" if kind == "dev" else ""), LFK_TEST_HOOKS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(mport), "-m", "llama_fastapi_k8s_gpu_amd.serve"]
    log = open(tmp_path / "serve.log", "w")
    proc = subprocess.Popen(cmd, env=env, cwd=root, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        t0, st = time.time(), None
        while time.time() - t0 < 200 and proc.poll() is None:
            try:
                st, h = _get(f"http://127.0.0.1:{port}/health")
                if st == 200:
                    break
            except Exception:
                pass
            time.sleep(1.0)
        assert st == 200, open(tmp_path / "serve.log").read()[-4000:]
        # the fault lands inside the first generation (command 4: its prefill + a few steps)
        codes = []
        for _ in range(3):
            code, body = _post(f"http://127.0.0.1:{port}/response")
            codes.append((code, body))
            if code != 200:
                break
        code, body = codes[-1]
        assert code == 500, (codes, open(tmp_path / "serve.log").read()[-4000:])
        assert "Internal server error" in body["detail"] and "rank 1" in body["detail"], body
        # /health: unhealthy, naming the failed rank; the poisoned group refuses the next request
        st, h = _get(f"http://127.0.0.1:{port}/health")
        assert st == 503 and h["status"] == "unhealthy", h
        assert "rank 1" in (h["engine"].get("error") or ""), h
        code2, body2 = _post(f"http://127.0.0.1:{port}/response", timeout=60.0)
        assert code2 == 500 and ("poisoned" in body2["detail"] or "group fault" in body2["detail"]), body2
    finally:
        try:
            os.killpg(proc.pid, signal.SIGTERM)   # our own session: torchrun and its two ranks
            proc.wait(timeout=60)
        except Exception:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait(timeout=30)
        log.close()
