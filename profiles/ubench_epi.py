"""Microbenchmark (round 5): AMPBlock1 conv1 -> act2 at the narrow stages' C3 shapes (B = 32 utterances x 400
frames: C = 24 at 1024 samples per frame, C = 48 at 512), as two launches (itts_amp_conv_fwd conv-only +
itts_aa_snakebeta_fwd) vs one (itts_amp_conv_act_fwd); HIP events, median of 5 after 2 warm-ups."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "index-tts-dubbing_amd"))
from indextts import _hip  # noqa: E402
from indextts.utils.synthetic import kaiser_sinc_lowpass  # noqa: E402
from indextts.vocoder.bigvgan import _Conv, conv1d_taps  # noqa: E402


def timeit(fn, n=5):
    ts = []
    for i in range(n + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    lib = _hip.load()
    B = 32
    for C, T in ((24, 400 * 1024), (48, 400 * 512)):
        x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
        t2 = torch.empty_like(x)
        y = torch.empty_like(x)
        lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
        up = torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).float().cuda()
        la, lb = (torch.randn(C) * 0.3).cuda(), (torch.randn(C) * 0.3).cuda()
        s = _hip.stream_ptr()
        nbytes = B * T * C * 2
        for k, d in ((3, 1), (7, 3), (11, 5)):
            conv = _Conv(*conv1d_taps(torch.randn(C, C, k) / (C * k) ** 0.5, d), torch.randn(C) * 0.1, C, C, "cuda")

            def conv_only():
                _hip.check(lib.itts_amp_conv_fwd(x.data_ptr(), T * C, C, None, None, None, None, conv.w.data_ptr(),
                                                 conv.bias.data_ptr(), None, None, t2.data_ptr(), T * C, C,
                                                 lens.data_ptr(), B, T, C, C, conv.ntaps, conv.offs, 1.0, s), "c")

            def act():
                _hip.check(lib.itts_aa_snakebeta_fwd(t2.data_ptr(), y.data_ptr(), up.data_ptr(), up.data_ptr(),
                                                     la.data_ptr(), lb.data_ptr(), lens.data_ptr(), B, C, T, T * C, C, 1,
                                                     T * C, C, 1, _hip.BF16, _hip.BF16, s), "a")

            def fused():
                _hip.check(lib.itts_amp_conv_act_fwd(x.data_ptr(), T * C, C, conv.w.data_ptr(), conv.bias.data_ptr(),
                                                     y.data_ptr(), T * C, C, lens.data_ptr(), B, T, C, C, conv.ntaps,
                                                     conv.offs, up.data_ptr(), up.data_ptr(), la.data_ptr(),
                                                     lb.data_ptr(), s), "f")
            tc, ta, tf = timeit(conv_only), timeit(act), timeit(fused)
            print(f"C={C} k={k} d={d}: conv {tc:7.1f} us ({2 * nbytes / tc / 1e3:5.0f} GB/s)  act {ta:7.1f} us "
                  f"({2 * nbytes / ta / 1e3:5.0f})  sum {tc + ta:7.1f}  | fused {tf:7.1f} us "
                  f"({2 * nbytes / tf / 1e3:5.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
