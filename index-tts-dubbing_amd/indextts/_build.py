"""Build libitts_hip.so in-tree with hipcc for gfx950 (no cmake/ninja needed).

Each ``csrc/*.hip`` compiles to its own object (in parallel, only when it or a header changed),
then one ``hipcc -shared`` link.  Used by ``__graft_entry__.build()``; also runnable as
``python -m indextts._build [--force]``.  ``ITTS_HIPCC_DEFS="-DX=1 ..."`` and ``ITTS_BUILD_OUT=path``
build an experiment variant next to the product library (microbenchmarks load it via
``ITTS_HIP_LIB``).
"""
from __future__ import annotations

import glob
import os
import shlex
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(PKG_DIR), "csrc")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(PKG_DIR)), "include")
OUT = os.path.join(PKG_DIR, "libitts_hip.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def needs_rebuild(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in sources() + _headers())


def build(force: bool = False, verbose: bool = True, out: str = None) -> str:
    out = out or os.environ.get("ITTS_BUILD_OUT", OUT)
    defs = shlex.split(os.environ.get("ITTS_HIPCC_DEFS", ""))
    if not force and not needs_rebuild(out):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tag = "".join(c if c.isalnum() else "_" for c in " ".join(defs))[:80] or "default"
    objdir = os.path.join(os.path.dirname(PKG_DIR), "build", ARCH + "_" + tag)
    os.makedirs(objdir, exist_ok=True)
    hdr_t = max([os.path.getmtime(h) for h in _headers()] + [0.0])

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(src), hdr_t):
            return obj
        cmd = [hipcc, f"--offload-arch={ARCH}", *FLAGS, *defs, "-I", CSRC, "-I", INCLUDE, "-c", src, "-o", obj + ".tmp"]
        if verbose:
            print("[itts build]", os.path.basename(src), " ".join(defs), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        return obj

    jobs = max(1, min(len(sources()), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources()))
    tmp = out + ".tmp"
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs], check=True)
    os.replace(tmp, out)
    if verbose:
        print("[itts build] linked", out, flush=True)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
