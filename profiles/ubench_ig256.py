"""igemm256 on the latent-pass GEMM shapes (M = 15488 packed rows at C3) through itts_igemm_fwd: HIP-event
time per launch, TFLOP/s, and the max relative error against a torch f32 matmul of the same bf16 operands
(load another build with ITTS_HIP_LIB for A/B).  Shapes: c_attn (K 1024, N 3072, f32 out), attn.c_proj and
mlp.c_proj (N 1024, f32 out with the residual), c_fc (N 4096, bf16 out, gelu)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch

from indextts import _hip
from indextts.vocoder.bigvgan import pack_taps

lib = _hip.load()
M = int(os.environ.get("M", "15488"))
REPS = int(os.environ.get("REPS", "20"))
torch.manual_seed(0)
shapes = [(1024, 3072, torch.float32, 0, False), (1024, 1024, torch.float32, 0, True),
          (1024, 4096, torch.bfloat16, 1, False), (4096, 1024, torch.float32, 0, True)]
tot_ms = 0.0
for K, N, odt, gelu, resid in shapes:
    A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    wt = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda") * 0.1
    wp = pack_taps([wt.float().cpu()], K, N).cuda()
    Y = torch.zeros(M, N, device="cuda", dtype=odt)
    Y0 = (torch.randn(M, N, device="cuda") * 0.1).to(odt) if resid else None

    def run():
        if resid:
            Y.copy_(Y0)
        _hip.check(lib.itts_igemm_fwd(A.data_ptr(), M * K, K, wp.data_ptr(), bias.data_ptr(), None,
                                      Y.data_ptr() if resid else None, None, Y.data_ptr(), M * N, N, None, 1, M,
                                      K, N, 1, _hip.i32_array([0]), 1, 0, 1.0, gelu, _hip.dtype_code(Y),
                                      _hip.stream_ptr()), "itts_igemm_fwd")
    run()
    torch.cuda.synchronize()
    ref = A.float() @ wt.float().t() + bias
    if gelu:
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    if resid:
        ref = ref + Y0.float()
    err = ((Y.float() - ref).abs().max() / ref.abs().max()).item()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(REPS)]
    for e0, e1 in ev:
        if resid:
            Y.copy_(Y0)
        e0.record()
        _hip.check(lib.itts_igemm_fwd(A.data_ptr(), M * K, K, wp.data_ptr(), bias.data_ptr(), None,
                                      Y.data_ptr() if resid else None, None, Y.data_ptr(), M * N, N, None, 1, M,
                                      K, N, 1, _hip.i32_array([0]), 1, 0, 1.0, gelu, _hip.dtype_code(Y),
                                      _hip.stream_ptr()), "itts_igemm_fwd")
        e1.record()
    torch.cuda.synchronize()
    ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    ms = ts[len(ts) // 2]
    tot_ms += ms
    print(f"M={M} K={K} N={N} out={str(odt)[6:]} gelu={gelu} resid={int(resid)}: {ms * 1e3:8.1f} us "
          f"{2.0 * M * N * K / (ms * 1e-3) / 1e12:7.1f} TF/s  max rel err {err:.2e}", flush=True)
print(f"per layer (4 GEMMs): {tot_ms * 1e3:.1f} us")
