"""itts_igemm_fwd on the C3 shapes: latent-pass GEMMs (M = 32 x 484 rows) and BigVGAN stage 0-2 convs
(B = 32 utterances, 3/7/11 taps).  HIP events around 10 launches each -> TFLOP/s."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch
from indextts import _hip
from indextts.vocoder.bigvgan import pack_taps

lib = _hip.load()
dev = "cuda"


def run(B, T, Cin, Cout, taps, dil, out_dtype=torch.bfloat16, n=10):
    x = torch.randn(B, T, Cin, device=dev).to(torch.bfloat16)
    y = torch.empty(B, T, Cout, device=dev, dtype=out_dtype)
    w = pack_taps([torch.randn(Cout, Cin) * 0.02 for _ in range(taps)], Cin, Cout).to(dev)
    offs = _hip.i32_array([j * dil - dil * (taps - 1) // 2 for j in range(taps)])
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    bias = torch.zeros(Cout, device=dev)

    def f():
        _hip.check(lib.itts_igemm_fwd(x.data_ptr(), T * Cin, Cin, w.data_ptr(), bias.data_ptr(), None, None, None,
                                      y.data_ptr(), T * Cout, Cout, lens.data_ptr(), B, T, Cin, Cout, taps, offs, 1, 0,
                                      1.0, 0, _hip.dtype_code(y), _hip.stream_ptr()), "igemm")
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / n
    fl = 2.0 * B * T * Cin * Cout * taps
    return us, fl / (us * 1e-6) / 1e12


tot = 0.0
for name, args in [("latent c_attn", (1, 15488, 1024, 3072, 1, 1, torch.float32)),
                   ("latent c_proj", (1, 15488, 1024, 1024, 1, 1)), ("latent c_fc", (1, 15488, 1024, 4096, 1, 1)),
                   ("latent mlp.proj", (1, 15488, 4096, 1024, 1, 1)),
                   ("voc s0 k11", (32, 1600, 768, 768, 11, 5)), ("voc s0 k3", (32, 1600, 768, 768, 3, 1)),
                   ("voc s1 k11", (32, 6400, 384, 384, 11, 5)), ("voc s1 k7", (32, 6400, 384, 384, 7, 3)),
                   ("voc s2 k11", (32, 25600, 192, 192, 11, 5)), ("voc s2 k3", (32, 25600, 192, 192, 3, 1))]:
    us, tf = run(*args)
    tot += us
    print(f"{name:18s} {us:9.1f} us  {tf:7.1f} TF/s", flush=True)
print(f"sum {tot / 1e3:.2f} ms")
