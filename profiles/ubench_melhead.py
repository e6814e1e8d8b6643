"""mel_head GEMM of the decode step (32 rows, K = 1024) at N = 8194 (257 column tiles of 32 on 256
CUs) vs N = 8192 (256 tiles): per launch in a graph chain, weights from HBM (rotating copies)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd"), os.path.join(REPO, "profiles")]
import torch  # noqa: E402
from indextts import _hip  # noqa: E402
from indextts.gpt.engine import pack_skinny  # noqa: E402
from ubench_decode import graph_time, lib  # noqa: E402

B, K = 32, 1024
h = (torch.randn(B, K, device="cuda") * 0.5).to(torch.bfloat16)
for N in (8194, 8192, 8160, 8226):
    w0 = pack_skinny(torch.randn(N, K) * 0.02)
    nc = max(2, int(320e6 // w0.numel() // 2))
    wl = [w0.cuda() for _ in range(nc)]
    bias = torch.zeros(N, device="cuda")
    y = torch.empty(B, (N + 15) // 16 * 16, device="cuda")

    def run(i):
        _hip.check(lib.itts_decode_gemm(h.data_ptr(), K, wl[i % nc].data_ptr(), K, N, B, bias.data_ptr(), None, None,
                                        None, None, 0, 0, 0, y.data_ptr(), y.shape[1], 0, 0, 1, _hip.stream_ptr()),
                   "mel_head")
    print(f"mel_head N={N} ({(N + 31) // 32} tiles): {graph_time(run, reps=40, n=400):.2f} us", flush=True)
