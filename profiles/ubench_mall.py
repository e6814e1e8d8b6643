"""Does an Infinity-Cache (MALL) resident operand speed up the decode-step kernels?
Same kernels as ubench_decode.py, in a captured graph of back-to-back launches, with the weights /
KV rotating over > 256 MiB of copies (HBM) vs one copy (MALL / L2 resident)."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from ubench_decode import *  # noqa: F401,F403
from ubench_decode import _hip, lib, dev, B, D, graph_time, pack_skinny, torch


def main():
    res = {}
    h = torch.randn(32, 4 * D, device=dev).to(torch.bfloat16)
    ws = torch.zeros(8 * B * D * 4, device=dev)
    gemms = [("c_attn", 3 * D, D, 2, 2), ("c_proj", D, D, 8, 2), ("c_fc", 4 * D, D, 1, 0), ("mlp_proj", D, 4 * D, 8, 2)]
    for name, N, K, ks, epi in ([] if "attn" in sys.argv else gemms):
        w0 = pack_skinny(torch.randn(N, K) * 0.02)
        ncopy = max(2, int(320e6 // (N * K * 2)))
        wl = [w0.to(dev) for _ in range(ncopy)]
        y = torch.zeros(B, N, dtype=torch.bfloat16 if name == "c_fc" else torch.float32, device=dev)
        Y = ws if epi == 2 else y
        ldy = N if epi == 2 else y.stride(0)
        bias = torch.zeros(N, device=dev)
        for mode, nc in (("hbm", ncopy), ("mall", 1)):
            def f(i):
                w = wl[i % nc]
                _hip.check(lib.itts_decode_gemm(h.data_ptr(), K, w.data_ptr(), K, N, B, None if epi == 2 else bias.data_ptr(),
                                                None, None, None, None, 0, int(name == "c_fc"), epi, Y.data_ptr(), ldy,
                                                _hip.dtype_code(Y), B * N, ks, _hip.stream_ptr()), name)
            t = graph_time(f, reps=40, n=400)
            res[f"{name}_{mode}"] = (round(t, 2), round(N * K * 2 / t / 1e3, 1))
        del wl
    H, Smax = 16, int(os.environ.get("ITTS_UB_SMAX", "600"))
    NKV = 8
    kcs = [torch.randn(B, H, Smax, 64, device=dev).to(torch.bfloat16) for _ in range(NKV)]
    vcs = [torch.randn(B, H, Smax, 64, device=dev).to(torch.bfloat16) for _ in range(NKV)]
    kc = kcs[0]
    qkv = torch.randn(2 * B * 3 * D, device=dev)
    o = torch.zeros(32, D, dtype=torch.bfloat16, device=dev)
    pad = torch.zeros(B, dtype=torch.int32, device=dev)
    bq = torch.zeros(3 * D, device=dev)
    for S in (283, 450):
        t = torch.tensor([S - 1 - 82, 0, 0, 0], dtype=torch.int32, device=dev)
        for mode, nc in (("hbm", NKV), ("mall", 1)):
            def fa(i):
                _hip.check(lib.itts_attn_decode(qkv.data_ptr(), 3 * D, 2, B * 3 * D, bq.data_ptr(), kcs[i % nc].data_ptr(),
                                                vcs[i % nc].data_ptr(), kc.stride(0), kc.stride(1), Smax, pad.data_ptr(), 82,
                                                t.data_ptr(), o.data_ptr(), D, B, H, 1, 1, _hip.stream_ptr()), "attn")
            tt = graph_time(fa)
            res[f"attn_S{S}_{mode}"] = (round(tt, 2), round(B * H * S * 256 / tt / 1e3, 1))
    tst = torch.zeros(4, dtype=torch.int32, device=dev)
    res["advance"] = (round(graph_time(lambda i: lib.itts_step_advance(tst.data_ptr(), 0, _hip.stream_ptr())), 2), None)
    for k, v in res.items():
        print(f"{k:16s} {v[0]:8.2f} us  {'' if v[1] is None else str(v[1]) + ' GB/s'}", flush=True)


if __name__ == "__main__":
    main()
