import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd"), os.path.join(REPO, "profiles")]
import torch
from indextts import _hip
from ubench_decode import graph_time, lib, pack_skinny
D, H, Smax, NKV = 1024, 16, 600, 6
for B, S in ((32, 283), (64, 142), (128, 71), (32, 142), (32, 90), (128, 300), (96, 283)):
    kcs = [torch.randn(B, H, Smax, 64, device="cuda").to(torch.bfloat16) for _ in range(NKV)]
    vcs = [torch.randn(B, H, Smax, 64, device="cuda").to(torch.bfloat16) for _ in range(NKV)]
    qkv = torch.randn(2 * B * 3 * D, device="cuda")
    o = torch.zeros(max(B, 32), D, dtype=torch.bfloat16, device="cuda")
    pad = torch.zeros(B, dtype=torch.int32, device="cuda")
    bq = torch.zeros(3 * D, device="cuda")
    kvb = min(82, S - 2)
    t = torch.tensor([S - 1 - kvb, 0, 0, 0], dtype=torch.int32, device="cuda")
    def fa(i):
        _hip.check(lib.itts_attn_decode(qkv.data_ptr(), 3 * D, 2, B * 3 * D, bq.data_ptr(), kcs[i % NKV].data_ptr(),
                                        vcs[i % NKV].data_ptr(), kcs[0].stride(0), kcs[0].stride(1), Smax, pad.data_ptr(),
                                        kvb, t.data_ptr(), o.data_ptr(), D, B, H, 1, 1, _hip.stream_ptr()), "attn")
    tt = graph_time(fa)
    print(f"attn B={B} S={S}: {tt:.2f} us  {B * H * S * 256 / tt / 1e3:.0f} GB/s", flush=True)
    del kcs, vcs
# GEMM hot vs cold
h = torch.randn(32, 4 * D, device="cuda").to(torch.bfloat16)
y = torch.zeros(32, 4 * D, dtype=torch.bfloat16, device="cuda")
bias = torch.zeros(4 * D, device="cuda")
w = pack_skinny(torch.randn(4 * D, D) * 0.02).cuda()
def fc(i):
    _hip.check(lib.itts_decode_gemm(h.data_ptr(), D, w.data_ptr(), D, 4 * D, 32, bias.data_ptr(), None, None, None, None,
                                    0, 1, 0, y.data_ptr(), 4 * D, 1, 0, 1, _hip.stream_ptr()), "fc")
print(f"c_fc hot-cache: {graph_time(fc):.2f} us")
