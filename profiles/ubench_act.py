"""Activation1d kernel at the vocoder's stage shapes (C3: B=32 x 400 frames, channel-last bf16):
mean time of itts_aa_snakebeta_fwd per stage over N launches (HIP events), and HBM GB/s of its
algorithmic bytes (read + write, 2 B each).  ITTS_ACT_MFMA=0 selects the VALU kernel."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch
from indextts import _hip
from indextts.utils.synthetic import kaiser_sinc_lowpass

lib = _hip.load()
B, N = 32, int(os.environ.get("N", "20"))
shapes = [(768, 1600), (384, 6400), (192, 25600), (96, 102400), (48, 204800), (24, 409600)]
if len(sys.argv) > 1:
    shapes = [s for s in shapes if str(s[0]) in sys.argv[1:]]
f = torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).reshape(-1).cuda()
for C, T in shapes:
    g = torch.Generator().manual_seed(C)
    x = (torch.randn(B, T, C, generator=g) * 1.5).to("cuda", torch.bfloat16)
    y = torch.empty_like(x)
    la, lb = (torch.randn(C, generator=g) * 0.5).cuda(), (torch.randn(C, generator=g) * 0.5).cuda()
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    def run():
        _hip.check(lib.itts_aa_snakebeta_fwd(x.data_ptr(), y.data_ptr(), f.data_ptr(), f.data_ptr(), la.data_ptr(),
                                             lb.data_ptr(), lens.data_ptr(), B, C, T, T * C, C, 1, T * C, C, 1,
                                             _hip.BF16, _hip.BF16, _hip.stream_ptr()), "act")
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(N):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / N
    nb = 4.0 * B * T * C
    print(f"act C={C:4d} T={T:6d}: {us:8.1f} us  {nb / us / 1e3:7.1f} GB/s", flush=True)
