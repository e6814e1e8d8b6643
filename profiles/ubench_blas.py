"""hipBLASLt (torch.mm, bf16 in / bf16 out, f32 accumulate) on the latent-pass GEMM shapes, for
comparison with itts_igemm_fwd (profiles/ubench_latent.py)."""
import torch
M = 15488
for K, N in ((1024, 4096), (4096, 1024), (1024, 3072), (1024, 1024)):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.mm(a, w.t())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        torch.mm(a, w.t())
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f"M={M} K={K} N={N}: {us:7.1f} us  {2.0 * M * N * K / (us * 1e-6) / 1e12:7.1f} TF/s", flush=True)
