"""The container's tensor-parallel bootstrap, end to end on the one-GPU test box:
``torchrun --nproc-per-node 2 -m llama_fastapi_k8s_gpu_amd.serve`` exactly as
docker/entrypoint.sh starts it for a multi-GPU pod (gloo control group, the engine's own
collectives, rank 0 serving HTTP, rank 1 following), with TP_DEVICE=0 putting both ranks
on the one GPU and TP_COMM=ipc (RCCL refuses two ranks on one device)."""
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _get(url, timeout=5.0):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.status, json.loads(r.read())


@pytest.mark.timeout(300)
def test_torchrun_serve_two_ranks_one_gpu(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf
    path = write_synthetic_gguf("tiny-llama3-tp", str(tmp_path / "tp.gguf"), seed=4)
    port, mport = _free_port(), _free_port()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MODEL_PATH=path, SPLIT_MODE="row", TP_COMM="ipc", TP_DEVICE="0", HOST="127.0.0.1",
               PORT=str(port), N_CTX="256", N_BATCH="64", MAX_BATCH="3", SEED="5", PYTHONPATH=root)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(mport), "-m", "llama_fastapi_k8s_gpu_amd.serve"]
    log = open(tmp_path / "serve.log", "w")
    proc = subprocess.Popen(cmd, env=env, cwd=root, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        t0, health = time.time(), None
        while time.time() - t0 < 200:
            if proc.poll() is not None:
                break
            try:
                st, health = _get(f"http://127.0.0.1:{port}/health")
                if st == 200:
                    break
            except Exception:
                time.sleep(1.0)
        assert health is not None, open(tmp_path / "serve.log").read()[-4000:]
        assert health["engine"]["tp"] == 2, health
        body = {"bot_profile": {"name": "Mia.f", "appearance": "a, b, c, d"}, "user_profile": {"name": "u"},
                "context": [{"turn": "user", "message": "hello there"}]}
        req = urllib.request.Request(f"http://127.0.0.1:{port}/response", data=json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=120) as r:
                status, text = r.status, json.loads(r.read())["response"]
        except urllib.error.HTTPError as e:
            raise AssertionError(f"{e.code} {e.read()[:2000]!r}\n" + open(tmp_path / "serve.log").read()[-6000:])
        assert status == 200 and isinstance(text, str)
    finally:
        try:
            os.killpg(proc.pid, signal.SIGTERM)   # our own session: torchrun and its two ranks
            proc.wait(timeout=60)
        except Exception:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait(timeout=30)
        log.close()
