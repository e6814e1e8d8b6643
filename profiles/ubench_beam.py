"""Microbenchmark of itts_beam_candidates (96 rows = 32 utterances x 3 beams, V = 8194) per decoding
mode and top_k, for the product library and experiment variants (ITTS_HIP_LIB=path).
Usage: python profiles/ubench_beam.py [lib.so ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "index-tts-dubbing_amd"))
from indextts import _hip  # noqa: E402


def run(path):
    lib = _hip.load(path)
    K, R, V = 3, 96, 8194
    ldl = (V + 3) // 4 * 4
    g = torch.Generator().manual_seed(0)
    lg = (torch.randn(R, ldl, generator=g) * 3).cuda()
    sn = (torch.rand(R, ldl, generator=g) < 0.02).to(torch.uint8).cuda()
    bs = torch.randn(R).cuda()
    ts = torch.tensor([17, 0, 1234, 0], dtype=torch.int32).cuda()
    ck = torch.empty(R, 2 * K, device="cuda")
    cs = torch.empty_like(ck)
    ct = torch.empty(R, 2 * K, dtype=torch.int32, device="cuda")
    st = _hip.stream_ptr()
    out = []
    for name, ds, tk, tp in [("search", 0, 0, 1.0), ("sample k0", 1, 0, 1.0), ("sample k2", 1, 2, 1.0),
                             ("sample k10", 1, 10, 1.0), ("sample k30 p0.8", 1, 30, 0.8), ("sample k64", 1, 64, 1.0),
                             ("sample k100", 1, 100, 1.0), ("sample p0.8", 1, 0, 0.8)]:
        call = lambda: lib.itts_beam_candidates(lg.data_ptr(), ldl, V, sn.data_ptr(), bs.data_ptr(), ts.data_ptr(), 0,  # noqa: E731
                                                0, 8193, 10.0, ds, 1.0, tk, tp, K, ck.data_ptr(), cs.data_ptr(),
                                                ct.data_ptr(), R, st)
        for _ in range(10):
            _hip.check(call(), "itts_beam_candidates")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 200
        e0.record()
        for _ in range(n):
            call()
        e1.record()
        torch.cuda.synchronize()
        out.append(f"{name:18s} {e0.elapsed_time(e1) / n * 1e3:8.2f} us")
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2:  # one process per library (the ctypes library is loaded once per process)
        import subprocess
        for p in sys.argv[1:]:
            subprocess.run([sys.executable, __file__, p], check=True)
    else:
        p = sys.argv[1] if len(sys.argv) > 1 else None
        print(p or "product", flush=True)
        for line in run(p):
            print("  " + line, flush=True)
