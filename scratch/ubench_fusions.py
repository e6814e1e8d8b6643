"""A/B microbenchmark of the decode-step fusions at B=32 (graph replays, rotating weight/KV buffers):
attention + separate c_proj split-K GEMM vs the fused itts_attn_decode_proj, and the 32-column vs the
16-column decode GEMM for c_fc (+gelu) and mel_head."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd"), os.path.join(REPO, "profiles")]
import torch
from indextts import _hip
from indextts.gpt.engine import pack_skinny16
from ubench_decode import graph_time, lib, pack_skinny

D, H, Smax, NKV, B = 1024, 16, 600, 6, 32
h = torch.randn(32, 4 * D, device="cuda").to(torch.bfloat16)
for name, N, K, gelu in (("c_fc", 4 * D, D, 1), ("mel_head", 8194, D, 0)):
    W = torch.randn(N, K) * 0.02
    ncopy = max(2, int(320e6 // (N * K * 2)))
    w32 = [pack_skinny(W).cuda() for _ in range(ncopy)]
    w16 = [pack_skinny16(W).cuda() for _ in range(ncopy)]
    Np = (N + 15) // 16 * 16
    y = torch.zeros(32, Np, dtype=torch.bfloat16 if gelu else torch.float32, device="cuda")
    bias = torch.zeros(N, device="cuda")

    def g32(i):
        _hip.check(lib.itts_decode_gemm(h.data_ptr(), K, w32[i % ncopy].data_ptr(), K, N, B, bias.data_ptr(), None,
                                        None, None, None, 0, gelu, 0, y.data_ptr(), Np, _hip.dtype_code(y), 0, 1,
                                        _hip.stream_ptr()), name)

    def g16(i):
        _hip.check(lib.itts_decode_gemm16(h.data_ptr(), K, w16[i % ncopy].data_ptr(), K, N, B, bias.data_ptr(), gelu,
                                          y.data_ptr(), Np, _hip.dtype_code(y), _hip.stream_ptr()), name)

    t32, t16 = graph_time(g32, reps=40, n=400), graph_time(g16, reps=40, n=400)
    print(f"{name}: 32-col {t32:.2f} us, 16-col {t16:.2f} us ({N * K * 2 / t16 / 1e3:.0f} GB/s)", flush=True)
    del w32, w16

for S in (120, 283, 450):
    kcs = [torch.randn(B, H, Smax, 64, device="cuda").to(torch.bfloat16) for _ in range(NKV)]
    vcs = [torch.randn(B, H, Smax, 64, device="cuda").to(torch.bfloat16) for _ in range(NKV)]
    qkv = torch.randn(2 * B * 3 * D, device="cuda")
    o = torch.zeros(32, D, dtype=torch.bfloat16, device="cuda")
    pad = torch.zeros(B, dtype=torch.int32, device="cuda")
    bq = torch.zeros(3 * D, device="cuda")
    ws = torch.zeros(16 * B * D, device="cuda")
    wt = torch.randn(D, D) * 0.02
    wsk = pack_skinny(wt).cuda()
    wp = wt.t().contiguous().to(torch.bfloat16).cuda()
    kvb = min(82, S - 2)
    t = torch.tensor([S - 1 - kvb, 0, 0, 0], dtype=torch.int32, device="cuda")

    def attn(i):
        _hip.check(lib.itts_attn_decode(qkv.data_ptr(), 3 * D, 2, B * 3 * D, bq.data_ptr(), kcs[i % NKV].data_ptr(),
                                        vcs[i % NKV].data_ptr(), kcs[0].stride(0), kcs[0].stride(1), Smax,
                                        pad.data_ptr(), kvb, t.data_ptr(), o.data_ptr(), D, B, H, 1, 1,
                                        _hip.stream_ptr()), "attn")

    def both(i):
        attn(i)
        _hip.check(lib.itts_decode_gemm(o.data_ptr(), D, wsk.data_ptr(), D, D, B, None, None, None, None, None, 0, 0, 2,
                                        ws.data_ptr(), D, 0, B * D, 2, _hip.stream_ptr()), "c_proj")

    def fused(i):
        _hip.check(lib.itts_attn_decode_proj(qkv.data_ptr(), 3 * D, 2, B * 3 * D, bq.data_ptr(),
                                             kcs[i % NKV].data_ptr(), vcs[i % NKV].data_ptr(), kcs[0].stride(0),
                                             kcs[0].stride(1), Smax, pad.data_ptr(), kvb, t.data_ptr(), wp.data_ptr(),
                                             D, ws.data_ptr(), B * D, D, B, H, 1, None, 0, _hip.stream_ptr()), "fused")

    print(f"S={S}: attn {graph_time(attn):.2f} us, attn + c_proj {graph_time(both):.2f} us, "
          f"fused {graph_time(fused):.2f} us", flush=True)
    del kcs, vcs
