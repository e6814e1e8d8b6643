"""Build libitts_hip.so in-tree with hipcc for gfx950 (no cmake/ninja needed).

Used by ``__graft_entry__.build()``; also runnable as ``python -m indextts._build``.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(PKG_DIR), "csrc")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(PKG_DIR)), "include")
OUT = os.path.join(PKG_DIR, "libitts_hip.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def needs_rebuild() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(s) > t for s in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_rebuild():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = OUT + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", "-I", CSRC, "-I", INCLUDE,
           "-Wno-unused-result", "-o", tmp] + sources()
    if verbose:
        print("[itts build]", " ".join(os.path.basename(c) if c.endswith(".hip") else c for c in cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
