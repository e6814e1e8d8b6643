"""Microbenchmark of the GPT decode-step kernels in isolation (B=32, IndexTTS-1.5 shapes):
back-to-back launches of one kernel, HIP events around N launches -> us per launch (incl. boundary)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import numpy as np, torch
from indextts import _hip
from indextts.gpt.engine import pack_skinny

lib = _hip.load()
dev = "cuda"
B, D = 32, 1024
N_IT = 200


def timeit(fn, n=N_IT):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def graph_time(fn, n=N_IT, reps=20):
    """fn(i): launch variant i (rotating buffers so that the bytes come from HBM, not the MALL)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n // reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (n // reps * reps)


def main():
    res = {}
    h = torch.randn(32, 4 * D, device=dev).to(torch.bfloat16)
    ws = torch.zeros(8 * B * D * 4, device=dev)
    for name, N, K, ks, epi in [("c_attn", 3 * D, D, 2, 2), ("c_proj", D, D, 2, 2), ("c_fc", 4 * D, D, 1, 0),
                                ("mlp_proj", D, 4 * D, 8, 2), ("mel_head", 8194, D, 1, 0)]:
        w0 = pack_skinny(torch.randn(N, K) * 0.02)
        ncopy = max(2, int(320e6 // (N * K * 2)))
        wl = [w0.to(dev) for _ in range(ncopy)]
        y = torch.zeros(B, ((N + 15) // 16) * 16, dtype=torch.bfloat16 if name == "c_fc" else torch.float32, device=dev)
        Y = ws if epi == 2 else y
        ldy = N if epi == 2 else y.stride(0)
        bias = torch.zeros(N, device=dev)

        def f(i):
            w = wl[i % ncopy]
            _hip.check(lib.itts_decode_gemm(h.data_ptr(), K, w.data_ptr(), K, N, B, None if epi == 2 else bias.data_ptr(),
                                            None, None, None, None, 0, int(name == "c_fc"), epi, Y.data_ptr(), ldy,
                                            _hip.dtype_code(Y if epi != 2 else ws), B * N, ks, _hip.stream_ptr()), name)
        t = graph_time(f, reps=40, n=400)
        del wl
        res[name] = (round(t, 2), round(N * K * 2 / t / 1e3, 1))
    # attention at S = 283
    H, Smax = 16, 600
    NKV = 8
    kcs = [torch.randn(B, H, Smax, 64, device=dev).to(torch.bfloat16) for _ in range(NKV)]
    vcs = [torch.randn(B, H, Smax, 64, device=dev).to(torch.bfloat16) for _ in range(NKV)]
    kc = kcs[0]
    qkv = torch.randn(2 * B * 3 * D, device=dev)
    o = torch.zeros(32, D, dtype=torch.bfloat16, device=dev)
    pad = torch.zeros(B, dtype=torch.int32, device=dev)
    bq = torch.zeros(3 * D, device=dev)
    for S in (120, 283, 450):
        t = torch.tensor([S - 1 - 82, 0, 0, 0], dtype=torch.int32, device=dev)

        def fa(i):
            _hip.check(lib.itts_attn_decode(qkv.data_ptr(), 3 * D, 2, B * 3 * D, bq.data_ptr(), kcs[i % NKV].data_ptr(),
                                            vcs[i % NKV].data_ptr(),
                                            kc.stride(0), kc.stride(1), Smax, pad.data_ptr(), 82, t.data_ptr(), o.data_ptr(), D,
                                            B, H, 1, 1, _hip.stream_ptr()), "attn")
        tt = graph_time(fa)
        res[f"attn_S{S}"] = (round(tt, 2), round(B * H * S * 256 / tt / 1e3, 1))
    # reduce + LN
    x = torch.randn(B, D, device=dev)
    g1 = torch.ones(D, device=dev); b1 = torch.zeros(D, device=dev)
    hh = torch.zeros(32, D, dtype=torch.bfloat16, device=dev)
    for ns in (2, 8):
        def fr(i):
            _hip.check(lib.itts_residual_reduce_ln(x.data_ptr(), D, ws.data_ptr(), ns, B * D, D, b1.data_ptr(), hh.data_ptr(),
                                                   D, B, D, g1.data_ptr(), b1.data_ptr(), None, None, 1, _hip.stream_ptr()), "red")
        res[f"reduce_{ns}"] = (round(graph_time(fr), 2), None)
    # empty-ish kernel floor
    tst = torch.zeros(4, dtype=torch.int32, device=dev)
    res["advance"] = (round(graph_time(lambda i: lib.itts_step_advance(tst.data_ptr(), 0, _hip.stream_ptr())), 2), None)
    for k, v in res.items():
        print(f"{k:12s} {v[0]:8.2f} us  {'' if v[1] is None else str(v[1]) + ' GB/s'}")


if __name__ == "__main__":
    main()
