"""The host weight packers of the C ABI (itts_gpt_fold_ln / itts_gpt_pack_frag / itts_gpt_pack_qkv12,
csrc/gpt_pack.hip) against a torch restatement of the layouts the decode kernels read (CPU only: the
packers are host functions, callable without a GPU).  The bf16 weights, fragment orders and the u fold
terms are bit-exact; c = ln_b^T W + bias accumulates in double in both, in different orders, so it is
checked to 1 f32 ulp.  Reference tensors: HF Conv1D weights of GPT2Block (modeling_gpt2.py:246-306) as
UnifiedVoice holds them (gpt/model.py:255-281)."""
import ctypes

import pytest
import torch


def ref_pack(w_t, cols):
    """W^T [N, K] -> [N/cols][K/ks][64][8] bf16 (lane cols*q + r holds W^T[cols nt + r][ks s + 8q : +8])"""
    N, K = w_t.shape
    ks = 16 if cols == 32 else 32
    Np = (N + cols - 1) // cols * cols
    w = torch.zeros(Np, K, dtype=torch.float32)
    w[:N] = w_t.float()
    g = 64 // cols
    return w.reshape(Np // cols, cols, K // ks, g, 8).permute(0, 2, 3, 1, 4).contiguous().to(torch.bfloat16)


def ref_fold(w_io, bias, ln):
    w, bias = w_io.double(), bias.double()
    if ln is None:
        return w.t().float().to(torch.bfloat16), None, bias.float()
    g, b = ln[0].double(), ln[1].double()
    wp = (w * g[:, None]).t().float().to(torch.bfloat16)
    return wp, wp.double().sum(1).float(), (b @ w + bias).float()


def ref_qkv12(wp, u, c, D=1024):
    b = torch.arange(256)
    cl, j = b % 8, b // 8
    h = 2 * cl + j // 16
    i = 12 * (j % 16)[:, None] + torch.arange(12)[None, :]
    cols = (i // 64) * D + h[:, None] * 64 + i % 64
    w12 = wp[cols.reshape(-1)].reshape(256, 12, D // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
    return w12, torch.stack([u[cols], c[cols]], 1).contiguous()


@pytest.fixture(scope="module")
def lib():
    from indextts import _build, _hip
    _build.build(verbose=False)
    return _hip.load()


@pytest.mark.parametrize("cols", [16, 32])
@pytest.mark.parametrize("N,K", [(64, 96), (8194, 64), (40, 256)])
def test_pack_frag_matches_layout(lib, cols, N, K):
    from indextts.gpt.engine import pack_frag
    if K % (16 if cols == 32 else 32):
        pytest.skip("K not a multiple of the fragment step")
    g = torch.Generator().manual_seed(N + K + cols)
    w = torch.randn(N, K, generator=g) * 0.05
    got = pack_frag(w, cols)
    want = ref_pack(w, cols)
    assert got.shape == want.shape
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))
    # bf16 input packs the same bytes as its f32 source
    assert torch.equal(pack_frag(w.to(torch.bfloat16), cols).view(torch.int16), want.view(torch.int16))


@pytest.mark.parametrize("with_ln", [True, False])
def test_fold_ln_matches_restatement(lib, with_ln):
    from indextts.gpt.engine import fold_ln_weights
    g = torch.Generator().manual_seed(7)
    K, N = 256, 96
    w_io = torch.randn(K, N, generator=g) * 0.02
    bias = torch.randn(N, generator=g) * 0.1
    ln = (1.0 + 0.1 * torch.randn(K, generator=g), 0.05 * torch.randn(K, generator=g)) if with_ln else None
    out = fold_ln_weights(w_io, bias, ln, "cpu", keep_wt=True)
    wp, u, c = ref_fold(w_io, bias, ln)
    assert torch.equal(out["wt"].view(torch.int16), wp.view(torch.int16))
    assert torch.equal(out["w16"].view(torch.int16), ref_pack(wp.float(), 16).view(torch.int16))
    if with_ln:
        assert torch.equal(out["u"], u)  # sums of bf16 values: exact in double, any order
    ulp = torch.finfo(torch.float32).eps * c.abs().clamp(min=1e-30)
    assert bool(((out["c"] - c).abs() <= ulp).all())


def test_pack_qkv12_matches_restatement(lib):
    from indextts.gpt.engine import fold_ln_weights, pack_qkv12
    g = torch.Generator().manual_seed(11)
    D = 1024
    w_io = torch.randn(D, 3 * D, generator=g) * 0.02
    bias = torch.randn(3 * D, generator=g) * 0.1
    ln = (1.0 + 0.1 * torch.randn(D, generator=g), 0.05 * torch.randn(D, generator=g))
    wx = fold_ln_weights(w_io, bias, ln, "cpu", keep_wt=True)
    got = pack_qkv12(wx, 16)
    w12, uc = ref_qkv12(wx["wt"], wx["u_host"], wx["c_host"], D)
    assert torch.equal(got["w12"].view(torch.int16), w12.view(torch.int16))
    assert torch.equal(got["uc"], uc)


def test_packer_argument_errors(lib):
    buf = (ctypes.c_uint16 * 64)()
    assert lib.itts_gpt_pack_frag(buf, 0, 4, 8, 32, buf) != 0  # K not a multiple of 16
    assert b"multiple" in lib.itts_last_error()
    assert lib.itts_gpt_pack_frag(buf, 0, 4, 16, 24, buf) != 0
    assert lib.itts_gpt_pack_qkv12(buf, buf, buf, 512, 8, buf, buf) != 0
    assert lib.itts_gpt_fold_ln(buf, buf, buf, None, 4, 4, buf, buf, buf) != 0
