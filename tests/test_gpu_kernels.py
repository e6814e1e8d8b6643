"""GPU unit tests of individual GPT kernels through the C ABI vs. plain PyTorch fp32 references.

Tolerance: bf16 GEMM operands (the reference uses the same bf16-rounded operands) with f32
accumulation -> |err| <= 1e-2 * (|A| @ |W|^T) (+ bf16 output rounding for bf16 outputs)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _lib():
    from indextts import _hip
    return _hip, _hip.load()


@pytest.mark.parametrize("K,N,M", [(256, 96, 3), (256, 256, 1), (512, 512, 1), (1024, 3072, 32), (1024, 8194, 32),
                                   (4096, 1024, 32), (1024, 1024, 45), (1024, 1024, 96), (4096, 1024, 150)])
@pytest.mark.parametrize("mode", ["plain", "ln", "ln2", "resid", "split2", "split8", "gelu_bf16"])
def test_decode_gemm(K, N, M, mode):
    from indextts.gpt.engine import pack_skinny
    _hip, lib = _lib()
    if mode in ("ln", "ln2") and K > 1024:
        pytest.skip("LN prologue is for K <= 1024")
    ksplit = int(mode[-1]) if mode.startswith("split") else 1
    if ksplit > 1 and (K // 16) % ksplit:
        pytest.skip("K/16 not divisible by ksplit")
    torch.manual_seed(K + N + M)
    Mp = (M + 31) // 32 * 32
    W = torch.randn(N, K) / K ** 0.5
    bias = torch.randn(N) * 0.1
    wsk = pack_skinny(W).cuda()
    g1, b1 = torch.randn(K) * 0.1 + 1, torch.randn(K) * 0.1
    g2, b2 = torch.randn(K) * 0.1 + 1, torch.randn(K) * 0.1
    X = torch.randn(Mp, K) * 2 + 0.5
    Wq = W.to(torch.bfloat16).float()
    lnm = {"ln": 1, "ln2": 2}.get(mode, 0)
    if lnm:
        A = F.layer_norm(X[:M], (K,), g1, b1, 1e-5)
        if lnm == 2:
            A = F.layer_norm(A, (K,), g2, b2, 1e-5)
        a_dev = X.cuda()
    else:
        A = X[:M].to(torch.bfloat16).float()
        a_dev = X.to(torch.bfloat16).cuda()
    prod = A.to(torch.bfloat16).float() @ Wq.t()
    gelu = mode == "gelu_bf16"
    epi = 2 if ksplit > 1 else (1 if mode == "resid" else 0)
    Y0 = torch.randn(Mp, N)
    if epi == 2:
        Y = torch.zeros(ksplit, M, N).cuda()
        ref = prod
    else:
        ref = prod + bias
        if gelu:
            ref = F.gelu(ref, approximate="tanh")
        if epi == 1:
            ref = ref + Y0[:M]
        Y = Y0.clone().to(torch.bfloat16 if gelu else torch.float32).cuda()
    gd, bd, g2d, b2d = g1.cuda(), b1.cuda(), g2.cuda(), b2.cuda()
    biasd = bias.cuda()
    _hip.check(lib.itts_decode_gemm(a_dev.data_ptr(), K, wsk.data_ptr(), K, N, M,
                                    None if epi == 2 else biasd.data_ptr(),
                                    gd.data_ptr() if lnm else None, bd.data_ptr() if lnm else None,
                                    g2d.data_ptr() if lnm == 2 else None, b2d.data_ptr() if lnm == 2 else None,
                                    lnm, int(gelu), epi, Y.data_ptr(), N, _hip.dtype_code(Y), M * N, ksplit,
                                    _hip.stream_ptr()), "decode_gemm")
    torch.cuda.synchronize()
    got = Y.sum(0).cpu() if epi == 2 else Y[:M].float().cpu()
    assert torch.isfinite(got).all()
    scale = (A.abs() @ Wq.abs().t()) + 1e-3
    tol = (2e-2 if gelu else 1e-2) * scale + (1e-2 if gelu else 0)
    err = (got - ref).abs()
    assert bool((err <= tol).all()), float((err / scale).max())
    if epi != 2 and Mp > M:  # rows beyond M untouched
        assert torch.equal(Y[M:].float().cpu(), Y0[M:].to(Y.dtype).float())


@pytest.mark.parametrize("K,N,M,gelu", [(1024, 4096, 32, True), (1024, 8194, 32, False), (512, 96, 3, False),
                                        (1024, 1000, 45, True)])
def test_decode_gemm16(K, N, M, gelu):
    """16-column decode GEMM (c_fc + gelu -> bf16, mel_head -> f32) vs torch fp32 on the same
    bf16-rounded operands: |err| <= 1e-2 * (|A| @ |W|^T) (+ bf16 output rounding with gelu); rows
    beyond M untouched."""
    from indextts.gpt.engine import pack_skinny16
    _hip, lib = _lib()
    torch.manual_seed(K + N + M)
    Mp = (M + 31) // 32 * 32
    W = torch.randn(N, K) / K ** 0.5
    bias = torch.randn(N) * 0.1
    X = torch.randn(Mp, K)
    A = X[:M].to(torch.bfloat16).float()
    Wq = W.to(torch.bfloat16).float()
    ref = A @ Wq.t() + bias
    if gelu:
        ref = F.gelu(ref, approximate="tanh")
    Y0 = torch.randn(Mp, N)
    Y = Y0.clone().to(torch.bfloat16 if gelu else torch.float32).cuda()
    a_dev, w_dev, b_dev = X.to(torch.bfloat16).cuda(), pack_skinny16(W).cuda(), bias.cuda()
    _hip.check(lib.itts_decode_gemm16(a_dev.data_ptr(), K, w_dev.data_ptr(), K, N, M, b_dev.data_ptr(), int(gelu),
                                      Y.data_ptr(), N, _hip.dtype_code(Y), _hip.stream_ptr()), "decode_gemm16")
    torch.cuda.synchronize()
    got = Y[:M].float().cpu()
    assert torch.isfinite(got).all()
    scale = (A.abs() @ Wq.abs().t()) + 1e-3
    tol = (2e-2 if gelu else 1e-2) * scale + (1e-2 if gelu else 0)
    err = (got - ref).abs()
    assert bool((err <= tol).all()), float((err / scale).max())
    if Mp > M:
        assert torch.equal(Y[M:].float().cpu(), Y0[M:].to(Y.dtype).float())


@pytest.mark.parametrize("K,N,M", [(1024, 3072, 32), (1024, 4096, 45), (1024, 1024, 96), (4096, 1024, 32),
                                   (512, 96, 3), (1024, 3072, 160)])
@pytest.mark.parametrize("mode", ["fold", "fold_gelu_bf16", "plain", "resid"])
def test_decode_gemm16x(K, N, M, mode):
    """itts_decode_gemm16x vs torch fp32 on the same bf16 operands.
    fold: y = LN(a) @ W + bias computed as rstd * (a @ W' - mean * u) + c (W' = bf16(diag(g) W),
    row statistics of the bf16 rows of a): compared with exactly that expression in fp32 (|err| <=
    1e-2 * rstd * (|a| @ |W'|)) AND with the unfolded LN(a) @ W + bias within the bf16 weight
    rounding (2e-2 relative to the same scale); resid: x += a @ W^T + bias in place and
    xh = bf16(x); rows >= M untouched; M > 32 exercises the row-tile batching (weights read once)."""
    from indextts.gpt.engine import fold_ln_weights
    _hip, lib = _lib()
    torch.manual_seed(K * 7 + N + M)
    Mp = (M + 31) // 32 * 32
    W_io = torch.randn(K, N) / K ** 0.5  # HF Conv1D [in, out]
    bias = torch.randn(N) * 0.1
    g, b = torch.randn(K) * 0.1 + 1, torch.randn(K) * 0.1
    fold = mode.startswith("fold")
    wx = fold_ln_weights(W_io, bias, (g, b) if fold else None, "cuda")
    X = torch.randn(Mp, K) * 1.5 + 0.3
    A = X.to(torch.bfloat16).float()
    gelu = mode == "fold_gelu_bf16"
    out_bf16 = gelu
    if fold:
        Wp = (W_io * g[:, None]).to(torch.bfloat16).float()  # W' [K, N]
        mu = A[:M].mean(1, keepdim=True)
        var = (A[:M] ** 2).mean(1, keepdim=True) - mu ** 2
        rstd = torch.rsqrt(var + 1e-5)
        ref = rstd * (A[:M] @ Wp - mu * Wp.sum(0)) + (b @ W_io + bias)
        scale = rstd * (A[:M].abs() @ Wp.abs()) + 1e-3
        unfolded = F.layer_norm(A[:M], (K,), g, b, 1e-5) @ W_io + bias
    else:
        Wq = W_io.to(torch.bfloat16).float()
        ref = A[:M] @ Wq + bias
        scale = A[:M].abs() @ Wq.abs() + 1e-3
    if gelu:
        ref = F.gelu(ref, approximate="tanh")
    Y0 = torch.randn(Mp, N)
    xh0 = torch.randn(Mp, N).to(torch.bfloat16)
    if mode == "resid":
        ref = ref + Y0[:M]
        Y = Y0.clone().cuda()
        xh = xh0.clone().cuda()
    else:
        Y = Y0.clone().to(torch.bfloat16 if out_bf16 else torch.float32).cuda()
        xh = None
    a_dev = X.to(torch.bfloat16).cuda()
    _hip.check(lib.itts_decode_gemm16x(a_dev.data_ptr(), K, wx["w16"].data_ptr(), K, N, M, _hip.ptr(wx["c"]),
                                       _hip.ptr(wx["u"]), 1e-5, int(gelu), int(mode == "resid"), Y.data_ptr(), N,
                                       _hip.dtype_code(Y), _hip.ptr(xh), N, 8, _hip.stream_ptr()), "gemm16x")
    torch.cuda.synchronize()
    got = Y[:M].float().cpu()
    assert torch.isfinite(got).all()
    tol = 1e-2 * scale + (1e-2 if out_bf16 else 0)
    err = (got - ref).abs()
    assert bool((err <= tol).all()), float((err / scale).max())
    if fold and not gelu:
        assert bool(((got - unfolded).abs() <= 2e-2 * scale + 1e-3).all())
    if mode == "resid":
        assert torch.equal(xh[:M].cpu(), Y[:M].cpu().to(torch.bfloat16))
        if Mp > M:
            assert torch.equal(xh[M:].cpu(), xh0[M:])
    if Mp > M:
        assert torch.equal(Y[M:].float().cpu(), Y0[M:].to(Y.dtype).float())


@pytest.mark.parametrize("S", [8, 16])
def test_residual_reduce_ln_matches_torch(S):
    """x += bias + the S split partials in order (S = 16: one per head from itts_attn_decode_proj);
    h = LN2(LN1(x)) in bf16."""
    _hip, lib = _lib()
    torch.manual_seed(S)
    B, D = 32, 1024
    x = torch.randn(B, D)
    part = torch.randn(S, B, D)
    bias = torch.randn(D)
    g1, b1, g2, b2 = torch.randn(D) + 1, torch.randn(D), torch.randn(D) + 1, torch.randn(D)
    xd, pd = x.clone().cuda(), part.cuda()
    h = torch.zeros(B, D, dtype=torch.bfloat16).cuda()
    args = [t.cuda() for t in (bias, g1, b1, g2, b2)]
    _hip.check(lib.itts_residual_reduce_ln(xd.data_ptr(), D, pd.data_ptr(), S, B * D, D, args[0].data_ptr(),
                                           h.data_ptr(), D, B, D, args[1].data_ptr(), args[2].data_ptr(),
                                           args[3].data_ptr(), args[4].data_ptr(), _hip.BF16, _hip.stream_ptr()),
               "reduce")
    torch.cuda.synchronize()
    xr = x + bias + part.sum(0)
    hr = F.layer_norm(F.layer_norm(xr, (D,), g1, b1, 1e-5), (D,), g2, b2, 1e-5)
    torch.testing.assert_close(xd.cpu(), xr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(h.float().cpu(), hr, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("S,cache,nsplit", [(1, "bf16", 1), (37, "bf16", 3), (300, "bf16", 4), (1000, "bf16", 1),
                                            (300, "f32", 1), (513, "bf16", 2)])
def test_attn_decode_matches_torch(S, cache, nsplit):
    """One decode step: q/k/v = bias + sum of nsplit c_attn partial slabs; appends k/v at
    kv_base + t, then softmax(q k^T / 8 + pad mask) v over the cached prefix; vs torch fp32 on the
    same (cache-rounded) keys/values.  |err| <= 2e-2 (bf16 output rounding) / 1e-5 (f32)."""
    _hip, lib = _lib()
    torch.manual_seed(S)
    B, H, smax = 5, 16, S + 8
    D = 64 * H
    cdt = torch.bfloat16 if cache == "bf16" else torch.float32
    kc = (torch.randn(B, H, smax, 64) * 0.5).to(cdt)
    vc = torch.randn(B, H, smax, 64).to(cdt)
    parts = torch.randn(nsplit, B, 3 * D) / nsplit ** 0.5
    bias = torch.randn(3 * D) * 0.1 if nsplit > 1 else None
    qkv = bias.expand(B, -1).clone() if bias is not None else torch.zeros(B, 3 * D)
    for sp in range(nsplit):  # the kernel's summation order (bias first), so k/v rows compare exactly
        qkv = qkv + parts[sp]
    pad = torch.tensor([0, 3, 0, min(7, S - 1), 1], dtype=torch.int32).clamp(max=S - 1)
    kv_base, t = S - 1 - 2, 2  # new key lands at index S - 1
    kd, vd = kc.clone().cuda(), vc.clone().cuda()
    out = torch.zeros(B, D, dtype=cdt).cuda()
    tst = torch.tensor([t, 0, 0, 0], dtype=torch.int32).cuda()
    qkv_d, pad_d = parts.cuda(), pad.cuda()  # keep device temporaries alive until the kernel ran
    bias_d = bias.cuda() if bias is not None else None
    _hip.check(lib.itts_attn_decode(qkv_d.data_ptr(), 3 * D, nsplit, B * 3 * D, _hip.ptr(bias_d), kd.data_ptr(),
                                    vd.data_ptr(), kd.stride(0),
                                    kd.stride(1), smax, pad_d.data_ptr(), kv_base, tst.data_ptr(),
                                    out.data_ptr(), D, B, H, _hip.dtype_code(kd), _hip.dtype_code(out),
                                    _hip.stream_ptr()), "attn_decode")
    torch.cuda.synchronize()
    kidx = S - 1
    q = qkv[:, :D].view(B, H, 64)
    kn, vn = qkv[:, D:2 * D].view(B, H, 64), qkv[:, 2 * D:].view(B, H, 64)
    kr, vr = kc.float().clone(), vc.float().clone()
    kr[:, :, kidx], vr[:, :, kidx] = kn, vn  # the kernel uses the exact f32 new k/v for the new key
    ref = torch.zeros(B, H, 64)
    for b in range(B):
        p0 = int(pad[b])
        sc = torch.einsum("hd,hsd->hs", q[b], kr[b, :, p0:kidx + 1]) / 8.0
        ref[b] = torch.einsum("hs,hsd->hd", sc.softmax(-1), vr[b, :, p0:kidx + 1])
    got = out.float().cpu().view(B, H, 64)
    tol = 2e-2 if cache == "bf16" else 1e-5
    assert float((got - ref).abs().max()) <= tol * max(1.0, float(ref.abs().max()))
    # the cache row kidx now holds the new k/v (rounded to the cache dtype); nothing else changed
    assert torch.equal(kd[:, :, kidx].cpu(), kn.to(cdt)) and torch.equal(vd[:, :, kidx].cpu(), vn.to(cdt))
    keep = torch.ones(smax, dtype=torch.bool)
    keep[kidx] = False
    assert torch.equal(kd[:, :, keep].cpu(), kc[:, :, keep]) and torch.equal(vd[:, :, keep].cpu(), vc[:, :, keep])


def test_attn_decode_ignores_padding_and_future_cache_slots():
    """Cache slots that are not keys of the row (left padding before pad[b], slots after this step's
    key) may hold anything, NaN included (torch.empty caches): the output stays finite and equal to
    the reference over the row's own keys."""
    _hip, lib = _lib()
    torch.manual_seed(11)
    B, H, S, smax = 4, 16, 400, 480
    D = 64 * H
    kc = (torch.randn(B, H, smax, 64) * 0.5).to(torch.bfloat16)
    vc = torch.randn(B, H, smax, 64).to(torch.bfloat16)
    pad = torch.tensor([0, 5, 40, 1], dtype=torch.int32)
    kidx = S - 1
    for b in range(B):
        kc[b, :, : int(pad[b])] = float("nan")
        vc[b, :, : int(pad[b])] = float("nan")
    kc[:, :, kidx + 1:] = float("nan")
    vc[:, :, kidx + 1:] = float("inf")
    qkv = torch.randn(B, 3 * D)
    kd, vd, qd, pd = kc.clone().cuda(), vc.clone().cuda(), qkv.cuda(), pad.cuda()
    out = torch.zeros(B, D, dtype=torch.bfloat16).cuda()
    tst = torch.tensor([2, 0, 0, 0], dtype=torch.int32).cuda()
    _hip.check(lib.itts_attn_decode(qd.data_ptr(), 3 * D, 1, B * 3 * D, None, kd.data_ptr(), vd.data_ptr(),
                                    kd.stride(0), kd.stride(1), smax, pd.data_ptr(), kidx - 2, tst.data_ptr(),
                                    out.data_ptr(), D, B, H, _hip.BF16, _hip.BF16, _hip.stream_ptr()), "attn_decode")
    torch.cuda.synchronize()
    q = qkv[:, :D].view(B, H, 64)
    kr, vr = kc.float().clone(), vc.float().clone()
    kr[:, :, kidx], vr[:, :, kidx] = qkv[:, D:2 * D].view(B, H, 64), qkv[:, 2 * D:].view(B, H, 64)
    got = out.float().cpu().view(B, H, 64)
    assert bool(torch.isfinite(got).all())
    for b in range(B):
        p0 = int(pad[b])
        sc = torch.einsum("hd,hsd->hs", q[b], kr[b, :, p0:kidx + 1]) / 8.0
        ref = torch.einsum("hs,hsd->hd", sc.softmax(-1), vr[b, :, p0:kidx + 1])
        assert float((got[b] - ref).abs().max()) <= 2e-2 * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("S", [300, 700])
def test_attn_decode_row_bit_identical_alone_and_in_a_128_row_step(S):
    """The launcher loads 4 keys per group per round for >= 128-row steps (long-form chunks) and 12 for
    smaller ones; the online softmax advances in fixed 4-key chunks either way, so a row's output does
    not depend on the batch it was decoded in (S > 128 keys, one row alone vs the same
    row inside a 128-row step, bit for bit)."""
    _hip, lib = _lib()
    B, H, smax = 128, 16, S + 8
    D = 64 * H
    g = torch.Generator(device="cuda").manual_seed(S)
    kc = (torch.randn(B, H, smax, 64, generator=g, device="cuda") * 0.5).to(torch.bfloat16)
    vc = torch.randn(B, H, smax, 64, generator=g, device="cuda").to(torch.bfloat16)
    qkv = torch.randn(B, 3 * D, generator=g, device="cuda")
    pad = (torch.arange(B, device="cuda", dtype=torch.int32) * 7) % 41
    kv_base, t = S - 1 - 2, 2
    tst = torch.tensor([t, 0, 0, 0], dtype=torch.int32).cuda()

    def run(rows):
        kd, vd = kc[:rows].clone(), vc[:rows].clone()
        out = torch.zeros(rows, D, dtype=torch.bfloat16, device="cuda")
        _hip.check(lib.itts_attn_decode(qkv.data_ptr(), 3 * D, 1, B * 3 * D, None, kd.data_ptr(), vd.data_ptr(),
                                        kd.stride(0), kd.stride(1), smax, pad.data_ptr(), kv_base, tst.data_ptr(),
                                        out.data_ptr(), D, rows, H, _hip.BF16, _hip.BF16, _hip.stream_ptr()),
                   "attn_decode")
        torch.cuda.synchronize()
        return out.cpu()

    full, alone = run(128), run(3)
    assert torch.equal(full[:3], alone)


@pytest.mark.parametrize("S,rows", [(37, False), (300, False), (513, True)])
def test_attn_decode_proj_matches_torch(S, rows):
    """Attention with attn.c_proj fused (itts_attn_decode_proj): part[h][b] = o_h[b] @ W[64h : 64h+64]
    with o_h the head's f32 attention output and W the bf16 c_proj weight in HF Conv1D [in, out]
    order; vs torch fp32 on the same bf16 cache and weights: |err| <= 2e-3 * (|o| @ |W|) + 1e-5.  The
    lineage-table variant (rows=True, identity table) reads the same keys.  This step's k/v are
    appended to the cache as in itts_attn_decode."""
    _hip, lib = _lib()
    torch.manual_seed(S + 1)
    B, H, smax, nsplit = 5, 16, S + 8, 2
    D = 64 * H
    kc = (torch.randn(B, H, smax, 64) * 0.5).to(torch.bfloat16)
    vc = torch.randn(B, H, smax, 64).to(torch.bfloat16)
    parts = torch.randn(nsplit, B, 3 * D) / nsplit ** 0.5
    bias = torch.randn(3 * D) * 0.1
    qkv = bias.expand(B, -1).clone()
    for sp in range(nsplit):
        qkv = qkv + parts[sp]
    W = (torch.randn(D, D) / D ** 0.5).to(torch.bfloat16)  # [in, out]
    pad = torch.tensor([0, 3, 0, min(7, S - 1), 1], dtype=torch.int32).clamp(max=S - 1)
    kv_base, t = S - 1 - 2, 2
    kd, vd = kc.clone().cuda(), vc.clone().cuda()
    part = torch.full((H, B, D), float("nan")).cuda()
    tst = torch.tensor([t, 0, 0, 0], dtype=torch.int32).cuda()
    qkv_d, pad_d, bias_d, w_d = parts.cuda(), pad.cuda(), bias.cuda(), W.cuda()
    kvr = torch.arange(B, dtype=torch.int32)[:, None].expand(B, smax).contiguous().cuda() if rows else None
    _hip.check(lib.itts_attn_decode_proj(qkv_d.data_ptr(), 3 * D, nsplit, B * 3 * D, bias_d.data_ptr(), kd.data_ptr(),
                                         vd.data_ptr(), kd.stride(0), kd.stride(1), smax, pad_d.data_ptr(), kv_base,
                                         tst.data_ptr(), w_d.data_ptr(), D, part.data_ptr(), B * D, D, B, H,
                                         _hip.BF16, _hip.ptr(kvr), smax if rows else 0, _hip.stream_ptr()),
               "attn_decode_proj")
    torch.cuda.synchronize()
    kidx = S - 1
    q = qkv[:, :D].view(B, H, 64)
    kn, vn = qkv[:, D:2 * D].view(B, H, 64), qkv[:, 2 * D:].view(B, H, 64)
    kr, vr = kc.float().clone(), vc.float().clone()
    kr[:, :, kidx], vr[:, :, kidx] = kn, vn
    o = torch.zeros(B, H, 64)
    for b in range(B):
        p0 = int(pad[b])
        sc = torch.einsum("hd,hsd->hs", q[b], kr[b, :, p0:kidx + 1]) / 8.0
        o[b] = torch.einsum("hs,hsd->hd", sc.softmax(-1), vr[b, :, p0:kidx + 1])
    Wf = W.float().view(H, 64, D)
    ref = torch.einsum("bhd,hdn->hbn", o, Wf)
    scale = torch.einsum("bhd,hdn->hbn", o.abs(), Wf.abs())
    got = part.cpu()
    assert torch.isfinite(got).all()
    err = (got - ref).abs()
    assert bool((err <= 2e-3 * scale + 1e-5).all()), float(err.max())
    assert torch.equal(kd[:, :, kidx].cpu(), kn.to(torch.bfloat16)) and torch.equal(vd[:, :, kidx].cpu(),
                                                                                     vn.to(torch.bfloat16))


@pytest.mark.parametrize("mode", ["bf16", "f32"])
def test_attn_prefill_matches_torch(mode):
    """Packed varlen causal attention with left padding (the prefill / latent-pass kernel): bf16
    mode runs the MFMA flash kernel (bf16 Q/K/V, f32 softmax), f32 mode the exact VALU kernel.
    vs torch fp32 on the same inputs: |err| <= 3e-2 (bf16) / 1e-4 (f32); the KV cache rows of every
    valid position are written (bf16: rounded)."""
    _hip, lib = _lib()
    torch.manual_seed(7)
    H, D = 16, 1024
    lens = [83, 200, 1, 130, 257]
    pads = [5, 0, 0, 17, 40]
    starts = [0]
    for n in lens[:-1]:
        starts.append(starts[-1] + n)
    M = sum(lens)
    qkv = torch.randn(M, 3 * D)
    smax = max(lens) + 4
    cdt = torch.bfloat16 if mode == "bf16" else torch.float32
    kc = torch.zeros(len(lens), H, smax, 64, dtype=cdt, device="cuda")
    vc = torch.zeros_like(kc)
    out = torch.zeros(M, D, dtype=cdt, device="cuda")
    qd = qkv.cuda()
    st_, ln_, pd_ = (torch.tensor(v, dtype=torch.int32, device="cuda") for v in (starts, lens, pads))
    _hip.check(lib.itts_attn_prefill(qd.data_ptr(), 3 * D, st_.data_ptr(), ln_.data_ptr(), pd_.data_ptr(), len(lens),
                                     max(lens), kc.data_ptr(), vc.data_ptr(), kc.stride(0), kc.stride(1),
                                     out.data_ptr(), D, H, _hip.dtype_code(kc), _hip.dtype_code(out),
                                     _hip.stream_ptr()), "attn_prefill")
    torch.cuda.synchronize()
    got = out.float().cpu()
    tol = 3e-2 if mode == "bf16" else 1e-4
    for i, (s0, n, p) in enumerate(zip(starts, lens, pads)):
        x = qkv[s0:s0 + n]
        q, k, v = (x[:, j * D:(j + 1) * D].view(n, H, 64).transpose(0, 1) for j in range(3))
        if mode == "bf16":
            q, k, v = ((q / 8).bfloat16().float() * 8, k.bfloat16().float(), v.bfloat16().float())
        sc = q @ k.transpose(1, 2) / 8.0
        mask = torch.ones(n, n, dtype=torch.bool).tril()
        mask[:, :p] = False
        sc = sc.masked_fill(~mask, float("-inf"))
        ref = (sc.softmax(-1).nan_to_num(0.0) @ v).transpose(0, 1).reshape(n, D)
        g = got[s0:s0 + n]
        assert float((g[p:] - ref[p:]).abs().max()) <= tol, (i, float((g[p:] - ref[p:]).abs().max()))
        kk = x[:, D:2 * D].view(n, H, 64).transpose(0, 1)
        # cache rows of every non-padding position (left-pad keys are never attended, not stored)
        torch.testing.assert_close(kc[i, :, p:n].float().cpu(), kk[:, p:].to(cdt).float(), rtol=0, atol=0)


def test_log_mel_kernel_matches_cpu_front_end():
    """itts_log_mel (direct DFT per frame on the GPU) vs the CPU MelSpectrogramFeatures restatement."""
    from indextts.utils.audio import MelSpectrogramFeatures, log_mel_hip
    g = torch.Generator().manual_seed(0)
    for L in (24000 // 3, 12345):
        x = 0.3 * torch.randn(2, L, generator=g)
        want = MelSpectrogramFeatures()(x)
        got = log_mel_hip(x.cuda()).cpu()
        assert got.shape == want.shape
        np.testing.assert_allclose(got.exp().numpy(), want.exp().numpy(), rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("orig", [44100, 16000, 22050, 48000])
def test_resample_kernel_matches_cpu_front_end(orig):
    """itts_resample_sinc vs the CPU restatement of torchaudio's sinc_interp_hann resampler (same
    float64-built table; f32 sums in tap order vs F.conv1d's order): |err| <= 2e-6 (signal ~0.3 rms)."""
    from indextts.utils.audio import resample, resample_hip
    g = torch.Generator().manual_seed(orig)
    x = 0.3 * torch.randn(2, orig // 3 + 17, generator=g)
    want = resample(x, orig, 24000)
    got = resample_hip(x.cuda(), orig, 24000).cpu()
    assert got.shape == want.shape
    assert float((got - want).abs().max()) <= 2e-6


@pytest.mark.parametrize("C,T", [(512, 511), (64, 40), (32, 7)])
def test_cond_subsample_matches_conv2d(C, T):
    """itts_cond_subsample vs F.conv2d(stride 2) + ReLU (Conv2dSubsampling2) in f32, read back in
    (t, f, c) order: |err| <= bf16 output rounding (2^-8 relative) + 1e-5."""
    from indextts.utils.hiplinear import HipLinearBank
    g = torch.Generator().manual_seed(C + T)
    mel = torch.randn(3, 100, T, generator=g) * 2 - 4
    sd = {"e.conv.0.weight": torch.randn(C, 1, 3, 3, generator=g) * 0.3, "e.conv.0.bias": torch.randn(C, generator=g)}
    bank = HipLinearBank({k: v.cuda() for k, v in sd.items()}, "cuda")
    got = bank.subsample(mel.cuda(), "e").float().cpu()
    want = F.relu(F.conv2d(mel.transpose(1, 2)[:, None], sd["e.conv.0.weight"], sd["e.conv.0.bias"], stride=2))
    want = want.permute(0, 2, 3, 1).reshape(3, want.shape[2], -1)  # [B, t, f * C] in (f, c) order
    assert got.shape == want.shape
    assert float(((got - want).abs() - want.abs() * 2 ** -8).max()) <= 1e-5


@pytest.mark.parametrize("C,T,K", [(512, 255, 15), (64, 9, 15), (36, 20, 5), (256, 37, 15), (768, 20, 7), (512, 5, 15)])
def test_cond_glu_dwconv_matches_torch(C, T, K):
    """itts_cond_glu_dwconv vs F.glu -> depthwise F.conv1d(padding K/2) -> LayerNorm -> SiLU in f32:
    |err| <= 1e-4 + bf16 output rounding."""
    from indextts.utils.hiplinear import HipLinearBank
    g = torch.Generator().manual_seed(C + T + K)
    a = torch.randn(2, T, 2 * C, generator=g)
    sd = {"m.depthwise_conv.weight": torch.randn(C, 1, K, generator=g) * 0.3,
          "m.depthwise_conv.bias": torch.randn(C, generator=g) * 0.1,
          "m.norm.weight": 1 + 0.1 * torch.randn(C, generator=g), "m.norm.bias": 0.1 * torch.randn(C, generator=g)}
    bank = HipLinearBank({k: v.cuda() for k, v in sd.items()}, "cuda")
    got = bank.glu_dwconv(a.cuda(), "m").float().cpu()
    bank.tiled = False
    assert float((bank.glu_dwconv(a.cuda(), "m").float().cpu() - got).abs().max()) <= 2e-2
    h = F.glu(a, dim=-1).transpose(1, 2)
    h = F.conv1d(h, sd["m.depthwise_conv.weight"], sd["m.depthwise_conv.bias"], padding=K // 2, groups=C)
    want = F.silu(F.layer_norm(h.transpose(1, 2), (C,), sd["m.norm.weight"], sd["m.norm.bias"], 1e-5))
    assert float(((got - want).abs() - want.abs() * 2 ** -8).max()) <= 1e-4


@pytest.mark.parametrize("M,K,N", [(8160, 25088, 512), (300, 4096, 96), (40, 2048, 512)])
def test_igemm_splitk_matches_linear(M, K, N):
    """itts_igemm_splitk (K in chunks as a batch of 1-tap GEMMs + fixed-order sum) vs F.linear on the
    bf16-rounded operands in f32: |err| <= 1e-4 * (|A| @ |W|^T) + 1e-5; equals the unsplit bank call
    within the same bound."""
    from indextts.utils.hiplinear import HipLinearBank
    g = torch.Generator().manual_seed(M + K)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g) * 0.1
    x = torch.randn(M, K, generator=g)
    bank = HipLinearBank({"l.weight": w.cuda(), "l.bias": b.cuda()}, "cuda")
    got = bank.splitk(x.cuda(), "l").cpu()
    xq, wq = x.to(torch.bfloat16).float(), w.to(torch.bfloat16).float()
    want = F.linear(xq, wq, b)
    bound = 1e-4 * (xq.abs() @ wq.abs().t()) + 1e-5
    assert bool(((got - want).abs() <= bound).all()), float((got - want).abs().max())
    assert bool(((bank(x.cuda(), "l").cpu() - got).abs() <= bound).all())


@pytest.mark.parametrize("B,T,H,lens", [(2, 255, 8, None), (3, 40, 2, [40, 17, 1]), (1, 70, 4, [0])])
def test_cond_rel_attn_matches_torch(B, T, H, lens):
    """itts_cond_rel_attn vs the f32 torch restatement of RelPositionMultiHeadedAttention
    (conditioning._rel_pos_mha's math: masked_fill(-inf), softmax, masked_fill(0)): |err| <= 2e-5."""
    import math
    _hip, lib = _lib()
    g = torch.Generator().manual_seed(B * T + H)
    C = 64 * H
    qkv = torch.randn(B, T, 3 * C, generator=g)
    pos = torch.randn(T, C, generator=g)
    u, v = torch.randn(H, 64, generator=g) * 0.3, torch.randn(H, 64, generator=g) * 0.3
    L = torch.tensor(lens if lens is not None else [T] * B, dtype=torch.int32)
    q, k, vv = qkv.split(C, -1)
    q = q.view(B, T, H, 64)
    k, vv = k.view(B, T, H, 64).transpose(1, 2), vv.view(B, T, H, 64).transpose(1, 2)
    pp = pos.view(1, T, H, 64).transpose(1, 2)
    sc = ((q + u).transpose(1, 2) @ k.transpose(-2, -1) + (q + v).transpose(1, 2) @ pp.transpose(-2, -1)) / math.sqrt(64)
    masked = (torch.arange(T)[None, :] >= L[:, None].long())[:, None, None, :]
    att = torch.softmax(sc.masked_fill(masked, float("-inf")), -1).masked_fill(masked, 0.0)
    want = (att @ vv).transpose(1, 2).reshape(B, T, C)
    out = torch.empty(B, T, C, device="cuda")
    qg, pg, ug, vg, lg = qkv.cuda(), pos.cuda(), u.cuda(), v.cuda(), L.cuda()
    _hip.check(lib.itts_cond_rel_attn(qg.data_ptr(), 3 * C, pg.data_ptr(), C, ug.data_ptr(), vg.data_ptr(),
                                      None if lens is None else lg.data_ptr(), B, T, H, 0.125, out.data_ptr(), C,
                                      _hip.F32, _hip.stream_ptr()), "rel_attn")
    got = out.cpu()
    assert float((got - want).abs().max()) <= 2e-5, float((got - want).abs().max())


@pytest.mark.parametrize("B,T,C,att", [(2, 511, 1536, True), (3, 37, 100, False), (1, 5, 64, True)])
def test_time_stats_matches_torch(B, T, C, att):
    """itts_time_stats vs the f32 torch restatement of ECAPA's _compute_statistics (softmax weights or
    uniform 1/T): |err| <= 1e-5 relative; row-independent (a batch's rows equal the rows alone)."""
    from indextts.utils.hiplinear import HipLinearBank
    g = torch.Generator().manual_seed(B * T + C)
    x = torch.randn(B, T, C, generator=g) * 2 + 0.5
    lg = torch.randn(B, T, C, generator=g) * 3 if att else None
    w = torch.softmax(lg, dim=1) if att else torch.full((1, T, 1), 1.0 / T)
    mean = (w * x).sum(1)
    std = torch.sqrt((w * (x - mean[:, None]) ** 2).sum(1).clamp(1e-12))
    bank = HipLinearBank({}, "cuda")
    gm, gs = bank.time_stats(x.cuda(), None if lg is None else lg.cuda())
    assert float(((gm.cpu() - mean).abs() / (mean.abs() + 1)).max()) <= 1e-5
    assert float(((gs.cpu() - std).abs() / (std.abs() + 1)).max()) <= 1e-5
    m1, s1 = bank.time_stats(x[-1:].cuda(), None if lg is None else lg[-1:].cuda())
    assert torch.equal(m1[0], gm[-1]) and torch.equal(s1[0], gs[-1])


@pytest.mark.parametrize("nk,masked", [(287, False), (100, True), (33, False)])
def test_cross_attn_matches_torch(nk, masked):
    """itts_cross_attn (PerceiverResampler attention, gpt/perceiver.py:111-150) vs torch fp32 on the same
    q / k / v: |err| <= 1e-5 relative to max|v|; masked keys excluded (the reference fills them with
    -finfo.max; the 32 latent keys are never masked); each prompt bit-identical alone and in a batch."""
    _hip, lib = _lib()
    g = torch.Generator().manual_seed(nk)
    B, H, n = 3, 8, 32
    inner = 64 * H
    q = torch.randn(B, n, inner, generator=g)
    kv = torch.randn(B, nk, 2 * inner, generator=g)
    km = torch.ones(B, nk, dtype=torch.bool)
    if masked:
        km[1, 60:] = False
        km[2, 40:] = False
    scale = 64 ** -0.5

    def run(qq, kvv, kmm):
        Bq = qq.shape[0]
        out = torch.empty(Bq, n, inner, device="cuda")
        qd, kd, md = qq.contiguous().cuda(), kvv.contiguous().cuda(), kmm.to(torch.uint8).contiguous().cuda()
        _hip.check(lib.itts_cross_attn(qd.data_ptr(), n * inner, inner, kd.data_ptr(), kd.data_ptr() + 4 * inner,
                                       nk * 2 * inner, 2 * inner, md.data_ptr(), Bq, n, nk, H, scale, out.data_ptr(),
                                       n * inner, inner, _hip.stream_ptr()), "cross_attn")
        torch.cuda.synchronize()
        return out.cpu()

    got = run(q, kv, km)
    k, v = kv.chunk(2, -1)
    qh = q.view(B, n, H, 64).transpose(1, 2)
    kh = k.reshape(B, nk, H, 64).transpose(1, 2)
    vh = v.reshape(B, nk, H, 64).transpose(1, 2)
    sim = (qh @ kh.transpose(-2, -1)) * scale
    sim = sim.masked_fill(~km[:, None, None, :], -torch.finfo(sim.dtype).max)
    ref = (sim.softmax(-1) @ vh).transpose(1, 2).reshape(B, n, inner)
    assert float((got - ref).abs().max()) <= 1e-5 * float(v.abs().max())
    one = run(q[1:2], kv[1:2], km[1:2])
    assert torch.equal(one[0], got[1])
