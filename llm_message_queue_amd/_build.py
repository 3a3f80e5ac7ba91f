"""In-tree native build (no setuptools/hipify): g++ for host C++ modules,
hipcc --offload-arch=gfx950 for the HIP kernel module.

Outputs land in ``llm_message_queue_amd/_lib/`` so they travel with the repo
snapshot to the GPU box (``*.so`` is git-ignored, not gpurun-ignored).

    python -m llm_message_queue_amd._build          # build what is stale
    python -m llm_message_queue_amd._build --force  # rebuild everything
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "csrc")
LIB = os.path.join(HERE, "_lib")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("LLMQ_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> List[str]:
    import pybind11
    inc = [sysconfig.get_paths()["include"], pybind11.get_include()]
    return [f"-I{p}" for p in inc]


def _targets() -> Dict[str, dict]:
    k = os.path.join(CSRC, "kernels")
    return {
        "_mlq": dict(
            compiler="g++",
            sources=[os.path.join(CSRC, "queue", "mlq.cpp")],
            deps=[os.path.join(CSRC, "queue", "mlq_core.h")],
            flags=["-O3", "-std=c++17", "-fvisibility=hidden", "-pthread"],
            libs=[],
        ),
        "_shmring": dict(
            compiler="g++",
            sources=[os.path.join(CSRC, "queue", "shm_ring.cpp")],
            deps=[os.path.join(CSRC, "queue", "shm_ring.h"), os.path.join(CSRC, "queue", "shm_coll.h")],
            flags=["-O3", "-std=c++17", "-fvisibility=hidden", "-pthread"],
            libs=["-lrt"],
        ),
        "_ingress": dict(
            compiler="g++",
            sources=[os.path.join(CSRC, "ingress", "http_ingress.cpp")],
            deps=[os.path.join(CSRC, "queue", "shm_ring.h"), os.path.join(CSRC, "ingress", "guard.h")],
            flags=["-O3", "-std=c++17", "-fvisibility=hidden", "-pthread"],
            libs=["-lrt", "-lcrypto"],
        ),
        "_hipops": dict(
            compiler=os.path.join(ROCM, "bin", "hipcc"),
            sources=[os.path.join(k, "hipops.hip")],
            deps=[os.path.join(k, f) for f in sorted(os.listdir(k))
                  if f.endswith((".hip", ".h", ".hpp", ".cuh"))] if os.path.isdir(k) else [],
            flags=["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fvisibility=hidden",
                   "-mcode-object-version=5", "-Wno-unused-result",
                   "-Wno-unused-command-line-argument", "-ffp-contract=fast"],
            libs=[f"-L{ROCM}/lib", "-lamdhip64"],
        ),
        "_textcpu": dict(
            compiler="g++",
            sources=[os.path.join(CSRC, "text", "text_cpu.cpp")],
            deps=[os.path.join(CSRC, "text", "text_cpu.h")],
            flags=["-O3", "-std=c++17", "-fvisibility=hidden", "-pthread"],
            libs=[],
        ),
        "_telemetry": dict(
            compiler="g++",
            sources=[os.path.join(CSRC, "telemetry", "telemetry.cpp")],
            deps=[],
            flags=["-O2", "-std=c++17", "-fvisibility=hidden", "-pthread",
                   f"-I{ROCM}/include"],
            libs=["-ldl"],   # libamd_smi is dlopen'ed at runtime (absent on CPU hosts)
        ),
    }


def _out(name: str) -> str:
    return os.path.join(LIB, name + EXT)


def _includes(path: str, seen: set) -> None:
    """Every in-tree header ``path`` includes, transitively (``#include "x"``
    resolved against the file's directory and ``csrc/``): the staleness check
    must not miss a header nobody listed (a stale ``_shmring`` once survived
    an edit of ``shm_coll.h``)."""
    import re
    try:
        with open(path, encoding="utf-8", errors="replace") as fh:
            text = fh.read()
    except OSError:
        return
    for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
        for base in (os.path.dirname(path), CSRC):
            cand = os.path.normpath(os.path.join(base, inc))
            if os.path.exists(cand):
                if cand not in seen:
                    seen.add(cand)
                    _includes(cand, seen)
                break


def _stale(name: str, t: dict) -> bool:
    out = _out(name)
    if not os.path.exists(out):
        return True
    mt = os.path.getmtime(out)
    deps = set(t["deps"])
    for src in t["sources"]:
        _includes(src, deps)
    return any(os.path.exists(s) and os.path.getmtime(s) > mt for s in list(t["sources"]) + sorted(deps))


def build_one(name: str, t: dict, verbose: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    out = _out(name)
    tmp = out + ".tmp"
    cmd = [t["compiler"], "-shared", "-fPIC"] + t["flags"] + _py_includes() + \
        [f"-I{CSRC}"] + t["sources"] + ["-o", tmp] + t["libs"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build of {name} failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    # a kernel whose host-side stub clang silently skipped (e.g. a target
    # builtin inside a lambda of a kernel template) links fine and fails only
    # at import on the GPU box: refuse it here
    if shutil.which("nm"):
        und = subprocess.run(["nm", "-D", "--undefined-only", tmp], capture_output=True, text=True).stdout
        stubs = [ln.split()[-1] for ln in und.splitlines() if "__device_stub__" in ln]
        if stubs:
            os.unlink(tmp)
            raise RuntimeError(f"native build of {name}: kernel stubs missing (host side dropped them): {stubs[:4]}")
    os.replace(tmp, out)
    return out


def build(force: bool = False, only: List[str] = None, verbose: bool = False) -> List[str]:
    todo = {n: t for n, t in _targets().items()
            if (only is None or n in only) and all(os.path.exists(s) for s in t["sources"])
            and (force or _stale(n, t))}
    if not todo:
        return []
    if shutil.which(_targets()["_hipops"]["compiler"]) is None and "_hipops" in todo:
        raise RuntimeError("hipcc not found; set ROCM_PATH")
    with ThreadPoolExecutor(max_workers=min(4, len(todo))) as ex:
        futs = {n: ex.submit(build_one, n, t, verbose) for n, t in todo.items()}
        return [f.result() for f in futs.values()]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", nargs="*")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    built = build(force=a.force, only=a.only, verbose=a.verbose)
    for b in built:
        print("built", os.path.relpath(b, ROOT))
    return 0


if __name__ == "__main__":
    sys.exit(main())
