"""Calibration workload for the FETCH_SIZE correction (the x2 gfx950 factor was applied
without a check).  Launches the c_fc-shaped decode GEMM (itts_decode_gemm16x: N = 4096, K = 1024,
M = 32, bf16 weights streamed with 16-B-per-lane non-temporal loads -- the access pattern whose bytes
traffic.py corrects) REPS times, each on its own weight copy (no MALL reuse), so the bytes each
dispatch must fetch are known: the 8,388,608 weight bytes + the 64 KiB A tile (read by every XCD:
<= 8 x 64 KiB) + the 32-column-tile biases.  ``profiles/traffic.py calibrate`` divides the measured
FETCH_SIZE by the weight bytes.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_c -o run -- python profiles/pmc_calibrate.py
    python profiles/traffic.py calibrate /tmp/pmc_c
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "index-tts-dubbing_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from indextts import _hip  # noqa: E402
from indextts.gpt.engine import pack_skinny16  # noqa: E402

N, K, M, REPS = 4096, 1024, 32, 24
WEIGHT_BYTES = N * K * 2


def main():
    lib = _hip.load()
    ws = [pack_skinny16(torch.randn(N, K) * 0.02).cuda() for _ in range(REPS)]
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    c = torch.zeros(N, device="cuda")
    y = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
    torch.cuda.synchronize()
    for w in ws:
        _hip.check(lib.itts_decode_gemm16x(a.data_ptr(), K, w.data_ptr(), K, N, M, c.data_ptr(), None, 1e-5, 1, 0,
                                           y.data_ptr(), N, _hip.BF16, None, 0, 8, _hip.stream_ptr()), "gemm16x")
    torch.cuda.synchronize()
    print(f"{REPS} dispatches of decode_gemm16x_kernel, {WEIGHT_BYTES} weight bytes each")


if __name__ == "__main__":
    main()
