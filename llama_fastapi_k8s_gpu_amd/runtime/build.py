"""Build the native extensions in-tree (no pip, no JIT cache):

  * ``_hip``  - gfx950 kernels + C++ engine + RCCL, compiled with ``hipcc
                --offload-arch=gfx950`` (HIP sources are written for CDNA4
                directly: no hipify, no CUDA shims);
  * ``_cpu``  - the C++ CPU backend (g++, OpenMP) for ``n_gpu_layers=0``.

Objects are cached by content hash under ``build/`` so rebuilding after a
one-file edit recompiles one file. ``python -m llama_fastapi_k8s_gpu_amd.runtime.build``
builds both.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(ROOT, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

HIP_SOURCES = ["kernels/gemv.hip", "kernels/attention.hip", "kernels/sampler.hip", "kernels/gemm.hip",
               "kernels/misc.hip", "kernels/bmm.hip",
               "kernels/moe.hip", "kernels/p2p_allreduce.hip"]
HOST_HIP_SOURCES = ["runtime/engine.cpp", "runtime/p2p.cpp", "runtime/scheduler.cpp",
                    "bindings_hip.cpp"]     # host code against the HIP runtime
HOST_SOURCES = ["runtime/gguf.cpp", "runtime/repack.cpp", "runtime/tp_channel.cpp"]          # plain C++ (+OpenMP)
CPU_SOURCES = ["cpu/cpu_backend.cpp", "runtime/gguf.cpp", "runtime/repack.cpp", "runtime/scheduler.cpp",
               "runtime/tp_channel.cpp", "bindings_cpu.cpp"]


def _includes() -> List[str]:
    import pybind11
    return ["-I" + CSRC, "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _local_includes(path: str, seen: set) -> None:
    """Every csrc header reachable from `path` through #include "..." (recursive)."""
    import re
    with open(path, "r", errors="replace") as fh:
        text = fh.read()
    for inc in re.findall(r'^\s*#\s*include\s*"([^"]+)"', text, flags=re.M):
        dep = os.path.normpath(os.path.join(os.path.dirname(path), inc))
        if not os.path.exists(dep):
            dep = os.path.normpath(os.path.join(CSRC, inc))
        if os.path.exists(dep) and dep not in seen:
            seen.add(dep)
            _local_includes(dep, seen)


def _hash(path: str, flags: List[str]) -> str:
    h = hashlib.sha1(" ".join(flags).encode())
    # the csrc headers this source includes (transitively): an edit to one of them
    # rebuilds its dependants and nothing else
    deps: set = set()
    _local_includes(path, deps)
    for dep in sorted(deps):
        h.update(dep.encode())
        with open(dep, "rb") as fh:
            h.update(fh.read())
    with open(path, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def _compile(cmd_prefix: List[str], src: str, flags: List[str]) -> str:
    path = os.path.join(CSRC, src)
    key = _hash(path, cmd_prefix + flags)
    obj = os.path.join(BUILD, src.replace("/", "_") + "." + key + ".o")
    if not os.path.exists(obj):
        os.makedirs(BUILD, exist_ok=True)
        tmp = f"{obj}.{os.getpid()}.tmp"  # concurrent builders (pytest-xdist) never share a temp
        cmd = cmd_prefix + flags + ["-c", path, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, obj)
    return obj


def hip_so_path() -> str:
    return os.path.join(OUT_DIR, "_hip" + EXT)


def cpu_so_path() -> str:
    return os.path.join(OUT_DIR, "_cpu" + EXT)


def build_hip(jobs: int = 8, verbose: bool = True) -> str:
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    inc = _includes()
    dev_flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
                 "-Wno-unused-result"] + inc
    host_hip_flags = ["-O3", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROCM, "include"),
                      "-Wno-unused-result"] + inc
    host_flags = ["-O3", "-fPIC", "-std=c++17", "-fopenmp", "-mavx2", "-mfma"] + inc
    clangxx = os.path.join(ROCM, "llvm", "bin", "clang++")
    jobs_list = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for s in HIP_SOURCES:
            jobs_list.append(ex.submit(_compile, [hipcc, "-x", "hip"], s, dev_flags))
        for s in HOST_HIP_SOURCES:
            jobs_list.append(ex.submit(_compile, [clangxx, "-x", "c++"], s, host_hip_flags))
        for s in HOST_SOURCES:
            jobs_list.append(ex.submit(_compile, ["g++"], s, host_flags))
        objs = [j.result() for j in jobs_list]
    out = hip_so_path()
    tmp = out + ".tmp"
    cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + \
          ["-L" + os.path.join(ROCM, "lib"), "-lrccl", "-lamdhip64", "-lrocprofiler-sdk-roctx", "-lgomp", "-Wl,-rpath," + os.path.join(ROCM, "lib")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    if verbose:
        print("built", out)
    return out


def build_cpu(jobs: int = 8, verbose: bool = True) -> str:
    flags = ["-O3", "-fPIC", "-std=c++17", "-fopenmp", "-mavx2", "-mfma", "-mf16c", "-DLFK_NO_HIP"] + _includes()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(["g++"], s, flags), CPU_SOURCES))
    out = cpu_so_path()
    tmp = out + ".tmp"
    cmd = ["g++", "-shared", "-fPIC", "-fopenmp", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    if verbose:
        print("built", out)
    return out


SANITIZE_SOURCES = ["cpu/cpu_backend.cpp", "runtime/gguf.cpp", "runtime/repack.cpp", "tools/sanitize_driver.cpp"]


def build_sanitize_driver(jobs: int = 4, verbose: bool = False) -> str:
    """Host-side ASan + UBSan build of the GGUF parser, repack and CPU engine with a
    small driver (device code cannot run under a GPU sanitizer on the pool)."""
    flags = ["-O1", "-g", "-std=c++17", "-fopenmp", "-mavx2", "-mfma", "-mf16c", "-DLFK_NO_HIP",
             "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined",
             "-I" + CSRC]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(["g++"], s, flags), SANITIZE_SOURCES))
    out = os.path.join(ROOT, "build", "sanitize_driver")
    tmp = f"{out}.{os.getpid()}.tmp"
    cmd = ["g++", "-fsanitize=address,undefined", "-fopenmp", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    if verbose:
        print("built", out)
    return out


def build_all(jobs: int = 8):
    return build_cpu(jobs), build_hip(jobs)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "cpu"):
        build_cpu()
    if which in ("all", "hip"):
        build_hip()
