"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer runs of the C++ runtime
(SURVEY 5.2 race/memory-safety tooling).

The GGUF parser, the planar repack and the CPU engine are built with
``-fsanitize=address,undefined`` into ``build/sanitize_driver``
(csrc/tools/sanitize_driver.cpp) and driven over

* the synthetic models end to end (parse, load, prefill, sampled decode), and
* deterministic mutations of a valid file (truncations and byte flips in the
  header / metadata / tensor-info region): every mutant must be parsed or
  rejected with a clean ``std::runtime_error`` -- never a sanitizer report, a
  crash or a hang.

GPU sanitizers (and XNACK-on code objects) are not available on the target pool,
so the device kernels are covered by the fp32-reference numerics tests instead.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from llama_fastapi_k8s_gpu_amd.gguf.synthetic import write_synthetic_gguf

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan/libubsan")

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")


@pytest.fixture(scope="module")
def driver():
    from llama_fastapi_k8s_gpu_amd.runtime.build import build_sanitize_driver
    try:
        return build_sanitize_driver()
    except RuntimeError as e:  # toolchain without the sanitizer runtimes
        pytest.skip(f"sanitizer build unavailable: {e}")


@pytest.fixture(scope="module")
def models(tmp_path_factory):
    d = tmp_path_factory.mktemp("san_models")
    names = ["tiny-llama3-q4_k_m", "tiny-mixtral-q4_k_m", "tiny-tinyllama-q8_0"]
    return {m: write_synthetic_gguf(m, str(d / f"{m}.gguf")) for m in names}


def _run(driver, *args, timeout=120):
    r = subprocess.run([driver, *map(str, args)], capture_output=True, text=True, env=ENV, timeout=timeout)
    report = r.stderr
    assert "AddressSanitizer" not in report and "runtime error:" not in report, report[-4000:]
    return r


@pytest.mark.parametrize("model", ["tiny-llama3-q4_k_m", "tiny-mixtral-q4_k_m", "tiny-tinyllama-q8_0"])
def test_engine_clean_under_asan_ubsan(driver, models, model):
    r = _run(driver, "run", models[model], 6)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "generated=6" in r.stdout


def _header_end(path):
    """Byte offset of the tensor data section (everything before it is parsed text)."""
    from llama_fastapi_k8s_gpu_amd.gguf.reader import GGUFReader
    rd = GGUFReader(path)
    return int(rd.data_offset)


def test_truncated_files_rejected_cleanly(driver, models, tmp_path):
    src = models["tiny-llama3-q4_k_m"]
    blob = open(src, "rb").read()
    hdr = _header_end(src)
    cuts = sorted({0, 3, 4, 8, 15, 23, 24, 31, hdr // 7, hdr // 3, hdr // 2, hdr - 1, hdr, hdr + 100, len(blob) - 1})
    for cut in cuts:
        p = tmp_path / f"cut{cut}.gguf"
        p.write_bytes(blob[:cut])
        r = _run(driver, "parse", p)
        assert r.returncode == 2, (cut, r.stdout, r.stderr)
        assert "rejected" in r.stdout


def test_mutated_headers_never_trip_sanitizers(driver, models, tmp_path):
    src = models["tiny-mixtral-q4_k_m"]
    blob = bytearray(open(src, "rb").read())
    hdr = _header_end(src)
    rng = np.random.default_rng(2024)
    outcomes = {0: 0, 2: 0}
    for i in range(40):
        m = bytearray(blob)
        for _ in range(int(rng.integers(1, 5))):
            pos = int(rng.integers(0, hdr))
            # flip to values that stress length / count / type fields
            m[pos] = int(rng.choice([0x00, 0xFF, 0x7F, 0x80, int(rng.integers(0, 256))]))
        p = tmp_path / f"mut{i}.gguf"
        p.write_bytes(bytes(m))
        r = _run(driver, "parse", p)
        assert r.returncode in (0, 2), (i, r.returncode, r.stdout, r.stderr[-2000:])
        outcomes[r.returncode] += 1
    assert outcomes[2] > 0  # the mutations do reach the rejection paths
