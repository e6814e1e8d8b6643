"""EXPERIMENT (needs the kernel of commit 1e98b38; removed again after this measurement): mlp.c_proj (K = 5120, N = 1280) at small row counts: split-K partials + the residual
reduce launch vs the last-arriver reduce inside the GEMM launch (itts_decode_gemm_reduce, commit
1e98b38), per launch in a graph chain; bit-identity of x / xh checked."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd"), os.path.join(REPO, "profiles")]
import torch  # noqa: E402
from indextts import _hip  # noqa: E402
from indextts.gpt.engine import pack_skinny  # noqa: E402
from ubench_decode import graph_time, lib  # noqa: E402

P, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
lib.itts_decode_gemm_reduce.argtypes = [P, I64, P, I32, I32, I32, P, P, I64, I64, I32, P, I64, P, I64, P, P]
D, K = 1280, 5120
torch.manual_seed(0)
w0 = pack_skinny(torch.randn(D, K) * 0.02)
ncopy = max(2, int(320e6 // (D * K * 2)))
wl = [w0.cuda() for _ in range(ncopy)]
bias = torch.randn(D, device="cuda") * 0.1
cnt = torch.zeros(64, dtype=torch.int32, device="cuda")
for B in [int(v) for v in os.environ.get("ROWS", "1,2,4,8,32").split(",")]:
    f = (torch.randn(B, K, device="cuda") * 0.5).to(torch.bfloat16)
    x0 = torch.randn(B, D, device="cuda")
    ws = torch.zeros(16 * B * D, device="cuda")

    def run_two(i, x, xh, ks):
        _hip.check(lib.itts_decode_gemm(f.data_ptr(), K, wl[i % ncopy].data_ptr(), K, D, B, None, None, None, None,
                                        None, 0, 0, 2, ws.data_ptr(), D, 0, B * D, ks, _hip.stream_ptr()), "gemm")
        _hip.check(lib.itts_residual_reduce_ln(x.data_ptr(), D, ws.data_ptr(), ks, B * D, D, bias.data_ptr(),
                                               xh.data_ptr(), D, B, D, None, None, None, None, 1, _hip.stream_ptr()),
                   "reduce")

    def run_one(i, x, xh, ks):
        _hip.check(lib.itts_decode_gemm_reduce(f.data_ptr(), K, wl[i % ncopy].data_ptr(), K, D, B, bias.data_ptr(),
                                               ws.data_ptr(), D, B * D, ks, x.data_ptr(), D, xh.data_ptr(), D,
                                               cnt.data_ptr(), _hip.stream_ptr()), "gemm_reduce")

    for ks in (4, 8):
        xa, xb = x0.clone(), x0.clone()
        ha = torch.zeros(B, D, dtype=torch.bfloat16, device="cuda")
        hb = ha.clone()
        for _ in range(3):
            run_two(0, xa, ha, ks)
            run_one(0, xb, hb, ks)
        torch.cuda.synchronize()
        same = bool(torch.equal(xa, xb) and torch.equal(ha, hb))
        xa2, ha2 = x0.clone(), ha.clone()
        t2 = graph_time(lambda i: run_two(i, xa2, ha2, ks), reps=40, n=400)
        t1 = graph_time(lambda i: run_one(i, xa2, ha2, ks), reps=40, n=400)
        print(f"mlp.c_proj rows={B} split-K {ks}: gemm+reduce {t2:.2f} us | in-launch reduce {t1:.2f} us | "
              f"bit-identical {same} counters-zero {int(cnt.abs().sum()) == 0}", flush=True)
