"""Decode-step tail kernels timed alone (HIP events over 200 back-to-back launches): mel_head on the
32-column decode GEMM at several N (8194 = 257 column tiles, 8192 = 256) and M, and the greedy token
selection + next embedding (itts_sample_embed) at B = 32 / 1."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch
from indextts import _hip
from indextts.gpt.engine import pack_skinny

lib = _hip.load()
dev = "cuda"
K, V = 1024, 8194
g = torch.Generator().manual_seed(0)
W = (torch.randn(V, K, generator=g) * 0.02)
wsk = pack_skinny(W).to(dev)
bias = torch.zeros(V, device=dev)
s = torch.cuda.current_stream().cuda_stream


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for M in (32, 1):
    a = torch.randn(32, K, generator=g).to(dev, torch.bfloat16)
    y = torch.empty(32, V + 6, device=dev)
    for N in (8194, 8192, 8160, 4096):
        f = lambda: _hip.check(lib.itts_decode_gemm(ctypes.c_void_p(a.data_ptr()), K, ctypes.c_void_p(wsk.data_ptr()), K, N, M,
                                                     ctypes.c_void_p(bias.data_ptr()), None, None, None, None, 0, 0, 0,
                                                     ctypes.c_void_p(y.data_ptr()), V + 6, 0, 0, 1, ctypes.c_void_p(s)),
                               "dg")
        print(f"mel_head decode_gemm M={M:2d} N={N}: {timeit(f):7.2f} us")

ldl = V + 6
emb = torch.randn(V, K, generator=g).to(dev)
pos = torch.randn(1024, K, generator=g).to(dev)
for B in (32, 1):
    logits = torch.randn(B, ldl, generator=g).to(dev)
    seen = torch.zeros(B, ldl, dtype=torch.uint8, device=dev)
    done = torch.zeros(B, dtype=torch.uint8, device=dev)
    codes = torch.zeros(B, 1024, dtype=torch.int32, device=dev)
    tstate = torch.tensor([5, 0, 0, 0], dtype=torch.int32, device=dev)
    x = torch.empty(B, K, device=dev)
    h = torch.empty(B, K, dtype=torch.bfloat16, device=dev)
    P = ctypes.c_void_p
    f = lambda: _hip.check(lib.itts_sample_embed(P(logits.data_ptr()), ldl, V, P(seen.data_ptr()), P(done.data_ptr()),
                                                 P(codes.data_ptr()), 1024, P(tstate.data_ptr()), 0, 0, 8193,
                                                 ctypes.c_float(10.0), P(emb.data_ptr()), P(pos.data_ptr()), 0, K, None,
                                                 None, P(x.data_ptr()), P(h.data_ptr()), 1, B, None, P(s)), "se")
    print(f"sample_embed B={B:2d}: {timeit(f):7.2f} us")
    f0 = lambda: _hip.check(lib.itts_sample_embed(P(logits.data_ptr()), ldl, V, P(seen.data_ptr()), P(done.data_ptr()),
                                                  P(codes.data_ptr()), 1024, P(tstate.data_ptr()), 0, 0, 8193,
                                                  ctypes.c_float(10.0), None, None, 0, K, None, None, None, None, 1, B,
                                                  None, P(s)), "se0")
    print(f"sample (no embedding) B={B:2d}: {timeit(f0):7.2f} us")
    z = torch.zeros(1, device=dev)
    fz = lambda: z.add_(1.0)
    print(f"empty elementwise launch: {timeit(fz):7.2f} us")
