"""The decode step's tail kernels at the IndexTTS-1.5 mel vocabulary (8194 ids = 256 x 32 + 2 columns):
mel_head on the 32-column decode GEMM (csrc/gpt_decode.hip) -- every column tile, the 2-column tail tile
included, bit-identical to computing it alone and within f32 rounding of torch, nothing stored past N -- and
the greedy token selection + next embedding (itts_sample_embed, csrc/gpt_sample.hip) equal to the HF
processors + argmax + mel_emb / mel_pos lookup (gpt/model.py:151-155, HF logits_process.py:409-412,
utils.py:2894-2925).  (Round 6 measured folding the 257th tile into the last workgroup and prefetching the
position row: both slower, profiles/tail_fold_r06x.txt; not kept.)"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
K, V = 1024, 8194


def _lib():
    from indextts import _hip
    return _hip, _hip.load()


def _dg(lib, hip, a, w, N, M, bias, y, ldy):
    s = torch.cuda.current_stream().cuda_stream
    hip.check(lib.itts_decode_gemm(a.data_ptr(), K, w, K, N, M, bias, None, None, None, None, 0, 0, 0, y.data_ptr(),
                                   ldy, 0, 0, 1, s), "itts_decode_gemm")


@pytest.mark.parametrize("M", [32, 7, 1])
def test_mel_head_tail_tile_bit_identical(M):
    from indextts.gpt.engine import pack_skinny
    hip, lib = _lib()
    g = torch.Generator().manual_seed(11 + M)
    W = torch.randn(V, K, generator=g) * 0.03
    b = torch.randn(V, generator=g) * 0.1
    wsk = pack_skinny(W).cuda()
    bias = b.cuda()
    a = torch.randn(32, K, generator=g).to("cuda", torch.bfloat16)
    ldy = V + 6
    full = torch.full((32, ldy), float("nan"), device="cuda")
    part = torch.full((32, ldy), float("nan"), device="cuda")
    _dg(lib, hip, a, wsk.data_ptr(), V, M, bias.data_ptr(), full, ldy)           # all 257 column tiles
    _dg(lib, hip, a, wsk.data_ptr(), 8192, M, bias.data_ptr(), part, ldy)        # tiles 0..255 alone
    tile = 256 * K * 32 * 2                                                      # bytes per 256 packed column tiles
    tail = torch.full((32, 8), float("nan"), device="cuda")
    _dg(lib, hip, a, wsk.data_ptr() + tile, 2, M, bias.data_ptr() + 8192 * 4, tail, 8)  # tile 256 alone
    torch.cuda.synchronize()
    assert torch.equal(full[:M, :8192], part[:M, :8192])
    assert torch.equal(full[:M, 8192:V], tail[:M, :2])
    assert torch.isnan(full[:M, V:]).all()  # nothing written past N
    ref = a[:M].float() @ W.cuda().to(torch.bfloat16).float().T + bias
    err = (full[:M, :V] - ref).abs().max().item()
    assert err < 2e-3 * ref.abs().max().item(), err


@pytest.mark.parametrize("B", [32, 1])
def test_sample_embed_greedy_matches_torch(B):
    hip, lib = _lib()
    g = torch.Generator().manual_seed(5 + B)
    ldl, ldc, stop, pen, col, pos_delta = V + 6, 64, 8193, 10.0, 9, 2
    logits = torch.randn(B, ldl, generator=g)
    seen = (torch.rand(B, ldl, generator=g) < 0.01).to(torch.uint8)
    seen[:, stop] = 0
    logits[0, 77] = 50.0
    seen[0, 77] = 1  # penalised: 50 / 10 = 5
    if B > 1:
        logits[1, stop] = 60.0  # min_new below the column: the stop id is masked
    done = torch.zeros(B, dtype=torch.uint8)
    emb = torch.randn(V, K, generator=g)
    pos = torch.randn(64, K, generator=g)
    tstate = torch.tensor([col, 0, 0, 0], dtype=torch.int32)
    d = {k: v.cuda() for k, v in dict(logits=logits, seen=seen.clone(), done=done, emb=emb, pos=pos,
                                        tstate=tstate).items()}
    codes = torch.zeros(B, ldc, dtype=torch.int32, device="cuda")
    x = torch.empty(B, K, device="cuda")
    h = torch.empty(B, K, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    hip.check(lib.itts_sample_embed(d["logits"].data_ptr(), ldl, V, d["seen"].data_ptr(), d["done"].data_ptr(),
                                    codes.data_ptr(), ldc, d["tstate"].data_ptr(), 0, col + 5, stop, pen,
                                    d["emb"].data_ptr(), d["pos"].data_ptr(), pos_delta, K, None, None, x.data_ptr(),
                                    h.data_ptr(), 1, B, None, s), "itts_sample_embed")
    torch.cuda.synchronize()
    sc = logits[:, :V].clone()
    pm = seen[:, :V].bool()
    sc[pm] = torch.where(sc[pm] < 0, sc[pm] * pen, sc[pm] / pen)
    sc[:, stop] = -float("inf")
    tok = sc.argmax(dim=1)
    assert torch.equal(codes[:, col].cpu().long(), tok)
    assert all(int(d["seen"][r, tok[r]]) == 1 for r in range(B))
    want_x = emb[tok] + pos[col + pos_delta]
    assert torch.equal(x.cpu(), want_x)
    assert torch.equal(h.cpu(), want_x.to(torch.bfloat16))
