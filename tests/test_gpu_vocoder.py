"""GPU parity of the BigVGAN2 HIP path (through the C ABI) against the CPU oracle / reference goldens.

Tolerances (stated per the north star: vocoder within fp tolerance):
  * Activation1d kernel, f32 in/out: max |err| <= 5e-5 (f32 math; accurate sinf)
  * implicit-GEMM conv, bf16 in / f32 out: max |err| <= 1e-4 * sum|w||x| (f32 accumulation of the
    same bf16-rounded operands)
  * full vocoder in bf16 storage vs the fp32 oracle: waveform relative RMS error <= 2e-2 and
    max |err| <= 0.05; int16 output == trunc(clamp(32767 * wav)) of the kernel's own wav exactly,
    and within ceil(32767 |wav - ref|) + 1 of the reference int16
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from parity_util import check_pcm, record, rel_rms

pytestmark = pytest.mark.gpu


def _lib():
    from indextts import _hip
    return _hip, _hip.load()


@pytest.mark.parametrize("i", range(5))
def test_activation_kernel_bct_matches_golden(golden, i):
    _hip, lib = _lib()
    x = torch.from_numpy(golden[f"act{i}_x"]).cuda()
    f = torch.from_numpy(golden[f"act{i}_filter"]).reshape(-1).cuda()
    a = torch.from_numpy(golden[f"act{i}_alpha"]).cuda()
    b = torch.from_numpy(golden[f"act{i}_beta"]).cuda()
    y = torch.empty_like(x)
    B, C, T = x.shape
    _hip.check(lib.itts_aa_snakebeta_bct(x.data_ptr(), y.data_ptr(), f.data_ptr(), f.data_ptr(), a.data_ptr(),
                                         b.data_ptr(), B, C, T, _hip.F32, _hip.stream_ptr()), "bct")
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.cpu().numpy(), golden[f"act{i}_y"], rtol=0, atol=5e-5)


def test_activation_kernel_ragged_channel_last():
    from oracle.bigvgan_oracle import activation1d
    from indextts.utils.synthetic import kaiser_sinc_lowpass
    _hip, lib = _lib()
    torch.manual_seed(0)
    B, T, C = 3, 301, 40
    lens = torch.tensor([301, 17, 2], dtype=torch.int32)
    x = torch.randn(B, T, C)
    f = torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).reshape(-1)
    la, lb = torch.randn(C) * 0.5, torch.randn(C) * 0.5
    xd, y = x.cuda(), torch.zeros(B, T, C, device="cuda")
    fd, lad, lbd, lensd = f.cuda(), la.cuda(), lb.cuda(), lens.cuda()
    _hip.check(lib.itts_aa_snakebeta_fwd(xd.data_ptr(), y.data_ptr(), fd.data_ptr(), fd.data_ptr(), lad.data_ptr(),
                                         lbd.data_ptr(), lensd.data_ptr(), B, C, T, T * C, C, 1, T * C, C, 1,
                                         _hip.F32, _hip.F32, _hip.stream_ptr()), "fwd")
    torch.cuda.synchronize()
    yc = y.cpu()
    for b in range(B):
        L = int(lens[b])
        ref = activation1d(x[b:b + 1, :L].transpose(1, 2), f, f, la, lb)[0].t()
        np.testing.assert_allclose(yc[b, :L].numpy(), ref.numpy(), rtol=0, atol=5e-5)


@pytest.mark.parametrize("C", [24, 48, 96, 192, 768])
def test_activation_kernel_bf16_mfma_path_vs_f32_path(C):
    """bf16 channel-last in / out (the vocoder's layout) runs both FIRs on MFMA (act_mfma.h) with the
    taps split into bf16 hi + lo and the SnakeBeta output rounded to bf16 before the down-sampler.
    vs the f32 VALU path on the same values: |d| <= 2^-7 |y| + 5e-3 rms(y) per element (one bf16 ulp
    of the output plus the 2^-9 rounding of the intermediate, which scales with |SnakeBeta(u)|, not
    |y|, carried through the 12-tap low-pass) and rms(d) <= 3e-3 rms(y) (the output rounding alone
    is ~1.1e-3);
    the 3 outputs at each utterance edge (VALU fix-up) are the f32 path rounded, bit for bit.
    Ragged rows cover a partial last time tile (len - t0 < tile), a row shorter than the filter
    halo (len < 6) and a one-sample row; rows >= len stay untouched."""
    from indextts.utils.synthetic import kaiser_sinc_lowpass
    _hip, lib = _lib()
    torch.manual_seed(C)
    B, T = 5, 1000  # >= 3 time tiles at every channel tile
    lens = torch.tensor([1000, 517, 5, 1, 263], dtype=torch.int32)
    x = (torch.randn(B, T, C) * 1.5).to(torch.bfloat16)
    f = torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).reshape(-1).cuda()
    la, lb = (torch.randn(C) * 0.5).cuda(), (torch.randn(C) * 0.5).cuda()
    lensd = lens.cuda()
    xb = x.cuda()
    xf = xb.float()
    sentinel = -12352.0  # exactly representable in bf16
    yb = torch.full((B, T, C), sentinel, dtype=torch.bfloat16, device="cuda")
    yf = torch.full((B, T, C), sentinel, dtype=torch.float32, device="cuda")
    for xin, yout, dt in ((xb, yb, _hip.BF16), (xf, yf, _hip.F32)):
        _hip.check(lib.itts_aa_snakebeta_fwd(xin.data_ptr(), yout.data_ptr(), f.data_ptr(), f.data_ptr(),
                                             la.data_ptr(), lb.data_ptr(), lensd.data_ptr(), B, C, T, T * C, C, 1,
                                             T * C, C, 1, dt, dt, _hip.stream_ptr()), "fwd")
    torch.cuda.synchronize()
    yb, yf = yb.cpu(), yf.cpu()
    rms = float(yf[0].pow(2).mean().sqrt())
    for b in range(B):
        L = int(lens[b])
        got, ref = yb[b, :L].float(), yf[b, :L]
        err = (got - ref).abs()
        bound = 2.0 ** -7 * ref.abs() + 5e-3 * rms
        assert bool((err <= bound).all()), (b, float((err - bound).max()))
        assert float(err.pow(2).mean().sqrt()) <= 3e-3 * rms, b
        edge = sorted({t for t in (0, 1, 2, L - 3, L - 2, L - 1) if 0 <= t < L})
        assert torch.equal(yb[b, edge].view(torch.int16), yf[b, edge].to(torch.bfloat16).view(torch.int16)), b
        assert bool((yb[b, L:].float() == sentinel).all()) and bool((yf[b, L:] == sentinel).all()), b
    # most outputs are the f32 path rounded exactly
    same = (yb[0].view(torch.int16) == yf[0].to(torch.bfloat16).view(torch.int16)).float().mean()
    assert float(same) > 0.6, float(same)


def test_activation_kernel_c96_whole_row_jobs_equal_block_jobs(monkeypatch):
    """C = 96 runs as ONE 3-block channel group per job (whole 192-B rows, ITTS_ACT_NB3=1, default) instead of
    three 1-block groups: the same per-channel-block MFMA arithmetic over the same window rows, so the
    outputs are bit-identical, ragged lengths included."""
    from indextts.utils.synthetic import kaiser_sinc_lowpass
    _hip, lib = _lib()
    C, B, T = 96, 40, 2100
    g = torch.Generator().manual_seed(C + B)
    lens = torch.randint(1, T + 1, (B,), generator=g, dtype=torch.int32)
    lens[0], lens[1], lens[2] = T, 1, 5
    x = (torch.randn(B, T, C, generator=g) * 1.5).to(torch.bfloat16).cuda()
    f = torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).reshape(-1).cuda()
    la, lb = (torch.randn(C, generator=g) * 0.5).cuda(), (torch.randn(C, generator=g) * 0.5).cuda()
    lensd = lens.cuda()
    out = []
    for nb3 in ("1", "0"):
        monkeypatch.setenv("ITTS_ACT_NB3", nb3)
        y = torch.full((B, T, C), -12352.0, dtype=torch.bfloat16, device="cuda")
        _hip.check(lib.itts_aa_snakebeta_fwd(x.data_ptr(), y.data_ptr(), f.data_ptr(), f.data_ptr(), la.data_ptr(),
                                             lb.data_ptr(), lensd.data_ptr(), B, C, T, T * C, C, 1, T * C, C, 1,
                                             _hip.BF16, _hip.BF16, _hip.stream_ptr()), "fwd")
        torch.cuda.synchronize()
        out.append(y.view(torch.int16).cpu())
    bad = (out[0] != out[1]).nonzero()
    assert bad.numel() == 0, (bad[:8].tolist(), lens.tolist())


@pytest.mark.parametrize("C,B,T", [(24, 160, 3000), (768, 64, 700), (192, 48, 1500), (96, 24, 2100)])
def test_activation_kernel_mfma_persistent_many_jobs(C, B, T):
    """The MFMA activation kernel is persistent (each workgroup walks several (utterance, time tile)
    jobs with the next window's loads in flight): shapes with more jobs than resident workgroups and
    ragged lengths (incl. empty tiles, a 1-sample and a 5-sample row) vs the f32 VALU path, same
    bound as above."""
    from indextts.utils.synthetic import kaiser_sinc_lowpass
    _hip, lib = _lib()
    g = torch.Generator().manual_seed(C + B)
    lens = torch.randint(1, T + 1, (B,), generator=g, dtype=torch.int32)
    lens[0], lens[1], lens[2] = T, 1, 5
    x = (torch.randn(B, T, C, generator=g) * 1.5).to(torch.bfloat16).cuda()
    f = torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).reshape(-1).cuda()
    la, lb = (torch.randn(C, generator=g) * 0.5).cuda(), (torch.randn(C, generator=g) * 0.5).cuda()
    lensd = lens.cuda()
    sentinel = -12352.0
    yb = torch.full((B, T, C), sentinel, dtype=torch.bfloat16, device="cuda")
    yf = torch.full((B, T, C), sentinel, dtype=torch.float32, device="cuda")
    for xin, yout, dt in ((x, yb, _hip.BF16), (x.float(), yf, _hip.F32)):
        _hip.check(lib.itts_aa_snakebeta_fwd(xin.data_ptr(), yout.data_ptr(), f.data_ptr(), f.data_ptr(),
                                             la.data_ptr(), lb.data_ptr(), lensd.data_ptr(), B, C, T, T * C, C, 1,
                                             T * C, C, 1, dt, dt, _hip.stream_ptr()), "fwd")
    torch.cuda.synchronize()
    yb, yf = yb.cpu(), yf.cpu()
    rms = float(yf[0].pow(2).mean().sqrt())
    for b in range(B):
        L = int(lens[b])
        err = (yb[b, :L].float() - yf[b, :L]).abs()
        assert bool((err <= 2.0 ** -7 * yf[b, :L].abs() + 5e-3 * rms).all()), b
        assert bool((yb[b, L:].float() == sentinel).all()), b


@pytest.mark.parametrize("i", range(5))
def test_activation_kernel_f16_bct(golden, i):
    """f16 in / f16 out through the reference op's argument list (the extension dispatches Half too,
    type_shim.h:20-43): within 1 f16 ulp of the f32 path on the same (f16-rounded) inputs rounded to
    f16 -- the arithmetic is f32 in both; the f16 store may fuse the last multiply-add into one
    rounding (v_fma_mix) where the f32 path rounds twice -- and within f16 rounding of the golden."""
    _hip, lib = _lib()
    x = torch.from_numpy(golden[f"act{i}_x"]).half().cuda()
    f = torch.from_numpy(golden[f"act{i}_filter"]).reshape(-1).cuda()
    a = torch.from_numpy(golden[f"act{i}_alpha"]).cuda()
    b = torch.from_numpy(golden[f"act{i}_beta"]).cuda()
    B, C, T = x.shape
    yh = torch.empty_like(x)
    xf = x.float()
    yf = torch.empty_like(xf)
    for xin, yout, dt in ((x, yh, _hip.F16), (xf, yf, _hip.F32)):
        _hip.check(lib.itts_aa_snakebeta_bct(xin.data_ptr(), yout.data_ptr(), f.data_ptr(), f.data_ptr(),
                                             a.data_ptr(), b.data_ptr(), B, C, T, dt, _hip.stream_ptr()), "bct")
    torch.cuda.synchronize()
    hb, fb = yh.cpu().view(torch.int16).int(), yf.cpu().half().view(torch.int16).int()
    assert int((hb - fb).abs().max()) <= 1 and bool(((hb < 0) == (fb < 0)).all())
    assert float((hb != fb).float().mean()) < 0.05
    ref = torch.from_numpy(golden[f"act{i}_y"])
    tol = 2e-3 * (ref.abs() + torch.from_numpy(golden[f"act{i}_x"]).abs().amax()) + 1e-3
    assert bool(((yh.cpu().float() - ref).abs() <= tol).all())
    # f16 in with a non-f16 out (or the reverse) is an argument error, nothing launched
    rc = lib.itts_aa_snakebeta_fwd(x.data_ptr(), yf.data_ptr(), f.data_ptr(), f.data_ptr(), a.data_ptr(),
                                   b.data_ptr(), None, B, C, T, C * T, 1, T, C * T, 1, T, _hip.F16, _hip.F32,
                                   _hip.stream_ptr())
    assert rc != 0 and b"f16" in lib.itts_last_error()


@pytest.mark.parametrize("cin,cout,k,d,T", [(768, 768, 3, 5, 150), (96, 96, 11, 3, 150), (24, 24, 7, 1, 150),
                                            (1024, 1536, 7, 1, 150), (12, 6, 3, 1, 150), (40, 200, 5, 2, 150),
                                            # Cout = 192: 256 x 64 window tiles (k >= 3), 128 x 64 at 1 tap;
                                            # several row tiles, a ragged second row
                                            (192, 192, 11, 5, 600), (192, 192, 3, 1, 600), (384, 192, 1, 1, 600),
                                            (768, 768, 7, 3, 600)])
def test_igemm_conv_matches_torch(cin, cout, k, d, T):
    from indextts.vocoder.bigvgan import _Conv, conv1d_taps
    _hip, lib = _lib()
    torch.manual_seed(cin + cout + k)
    B = 2
    lens = torch.tensor([T, T // 2 + 1], dtype=torch.int32)
    x = torch.randn(B, T, cin).to(torch.bfloat16)
    w = torch.randn(cout, cin, k) / (cin * k) ** 0.5
    bias = torch.randn(cout) * 0.1
    conv = _Conv(*conv1d_taps(w, d), bias, cin, cout, "cuda")
    y = torch.zeros(B, T, cout, device="cuda")
    xd, lensd = x.cuda(), lens.cuda()
    _hip.check(lib.itts_igemm_fwd(xd.data_ptr(), T * cin, cin, conv.w.data_ptr(), conv.bias.data_ptr(), None, None,
                                  None, y.data_ptr(), T * cout, cout, lensd.data_ptr(), B, T, cin, cout, conv.ntaps,
                                  conv.offs, 1, 0, 1.0, 0, _hip.F32, _hip.stream_ptr()), "igemm")
    torch.cuda.synchronize()
    wq = w.to(torch.bfloat16).float()
    for b in range(B):
        L = int(lens[b])
        ref = F.conv1d(x[b:b + 1, :L].float().transpose(1, 2), wq, bias, dilation=d, padding=d * (k - 1) // 2)[0].t()
        scale = F.conv1d(x[b:b + 1, :L].float().abs().transpose(1, 2), wq.abs(), dilation=d,
                         padding=d * (k - 1) // 2)[0].t()
        err = (y[b, :L].cpu() - ref).abs()
        assert bool((err <= 1e-4 * scale + 1e-5).all()), float(err.max())


def _vocoder(tag):
    from indextts.utils.config import load_config, default_config_path, tiny_config
    from indextts.utils.synthetic import bigvgan_state_dict
    from indextts.vocoder.bigvgan import HipBigVGAN
    from oracle.bigvgan_oracle import BigVGANOracle
    cfg = tiny_config() if tag == "tiny" else load_config(default_config_path())
    sd = bigvgan_state_dict(cfg.bigvgan, 0)
    return HipBigVGAN(sd, cfg.bigvgan, "cuda"), BigVGANOracle(sd, cfg.bigvgan)


@pytest.mark.parametrize("tag", ["tiny", "full"])
def test_vocoder_c_forward_equals_python_launches(tag):
    """itts_bigvgan_forward (the whole generator as one C-ABI call, bigvgan_fwd.hip) == the Python launch
    sequence of the same kernels (HipBigVGAN._forward_py), bit for bit: ragged batch (incl. a 1-frame
    utterance), random latents and speaker embeddings."""
    voc, _ = _vocoder(tag)
    g = torch.Generator().manual_seed(11)
    B, T = 3, 9 if tag == "tiny" else 6
    lat = (torch.randn(B, T, voc.conv_pre.cin, generator=g) * 0.5).to(torch.bfloat16).cuda()
    lens = torch.tensor([T, 1, T - 2], dtype=torch.int32)
    spk = torch.randn(B, voc._cond_w["cond_layer"].shape[1], generator=g).cuda()
    voc.cforward = True
    wav_c, pcm_c = voc.forward(lat, lens, spk)
    wav_p, pcm_p = voc._forward_py(lat, lens, spk)
    torch.cuda.synchronize()
    for b in range(B):
        n = int(lens[b]) * voc.hop
        assert torch.equal(wav_c[b, :n].cpu(), wav_p[b, :n].cpu()), b
        assert torch.equal(pcm_c[b, :n].cpu(), pcm_p[b, :n].cpu()), b


@pytest.mark.parametrize("tag", ["tiny", "full"])
def test_vocoder_matches_reference_golden(golden, tag):
    voc, _ = _vocoder(tag)
    lat = torch.from_numpy(golden[f"{tag}_bv_latent"]).cuda()
    spk = torch.from_numpy(golden[f"{tag}_bv_spk"]).cuda()
    wav, pcm = voc.forward(lat, torch.tensor([lat.shape[1]]), spk)
    torch.cuda.synchronize()
    ref = golden[f"{tag}_bv_wav"][:, 0]
    got = wav.cpu().numpy()
    rel = np.sqrt(np.mean((got - ref) ** 2) / np.mean(ref ** 2))
    record(f"vocoder_golden_{tag}", rel_rms=rel, max_abs=float(np.abs(got - ref).max()))
    # <= 1.5x the round-4 measurement (profiles/parity_r04d.json: tiny 8.4e-3 / 9.7e-3, full 1.01e-2 / 7.9e-3)
    bar_rel, bar_max = {"tiny": (1.3e-2, 0.015), "full": (1.55e-2, 0.012)}[tag]
    assert rel <= bar_rel, rel
    assert np.abs(got - ref).max() <= bar_max
    # int16: exactly the Q8 conversion of the kernel's own waveform; vs the reference's int16 at most
    # the scaled float error + 1 (was a flat 0.05 * 32767 LSB bound)
    check_pcm(got[0], pcm[0].cpu().numpy(), ref[0], golden[f"{tag}_bv_int16"][0, 0])


# stage-local bar: each stage's output vs the fp32 oracle stage fed the SAME bf16 stage input, so only
# that stage's own arithmetic (bf16 storage of its ~20 intermediate tensors, MFMA accumulation) is
# compared; an indexing / edge error inside one stage cannot hide under the end-to-end 2e-2 bar.
STAGE_REL = 5.5e-3   # measured r04 <= 3.6e-3: profiles/parity_r04d.json "vocoder_stage*" (1.5x)
EDGE_REL = 5.5e-3    # the first / last 64 output rows of every utterance (edge padding paths; measured <= 3.6e-3)


def test_vocoder_stage_local_parity():
    """Full IndexTTS-1.5 vocoder, ragged batch (12 and 7 frames): conv_pre, each of the 6 upsampling
    stages (ConvTranspose + speaker bias + mean of 3 AMPBlock1) and the post block checked one at a
    time against BigVGANOracle.pre / .stage / .post (models.py:201-250) run in fp32 on the kernel's own
    bf16 stage input, per utterance at its own length.  Bars: rel-RMS <= STAGE_REL over each stage,
    rel-RMS <= EDGE_REL over the 64 rows at each utterance end (vs the stage's RMS)."""
    voc, orc = _vocoder("full")
    g = torch.Generator().manual_seed(21)
    T, lens = 12, torch.tensor([12, 7], dtype=torch.int32)
    B = lens.numel()
    lat = (torch.randn(B, T, voc.conv_pre.cin, generator=g) * 0.5).to(torch.bfloat16)
    spk = torch.randn(B, voc._cond_w["cond_layer"].shape[1], generator=g)
    taps = {}
    wav, _ = voc._forward_py(lat.cuda(), lens, spk.cuda(), want_pcm=False, taps=taps)
    torch.cuda.synchronize()
    names = ["pre"] + [f"stage{i}" for i in range(len(voc.ups))]
    worst = {}
    for si, name in enumerate(names):
        out = taps[name].float().cpu()
        olen = taps[name + "_lens"].cpu()
        for b in range(B):
            n = int(olen[b])
            with torch.no_grad():
                if si == 0:
                    ref = orc.pre(lat[b:b + 1, : int(lens[b])].float(), spk[b:b + 1])
                else:
                    prev = taps[names[si - 1]].float().cpu()
                    m = int(taps[names[si - 1] + "_lens"][b])
                    ref = orc.stage(si - 1, prev[b:b + 1, :m].transpose(1, 2), spk[b:b + 1])
            ref = ref[0].transpose(0, 1).numpy()  # [n, C]
            got = out[b, :n].numpy()
            assert ref.shape == got.shape, (name, ref.shape, got.shape)
            r = rel_rms(got, ref)
            scale = np.sqrt(np.mean(ref.astype(np.float64) ** 2))
            e = min(64, n)
            edge = max(float(np.sqrt(np.mean((got[:e] - ref[:e]) ** 2))),
                       float(np.sqrt(np.mean((got[-e:] - ref[-e:]) ** 2)))) / scale
            worst[name] = max(worst.get(name, (0, 0))[0], r), max(worst.get(name, (0, 0))[1], edge)
            assert r <= STAGE_REL and edge <= EDGE_REL, (name, b, r, edge)
    # post block (activation_post -> conv_post -> tanh) on the last stage's bf16 output
    last = taps[names[-1]].float().cpu()
    for b in range(B):
        n = int(taps[names[-1] + "_lens"][b])
        with torch.no_grad():
            ref = orc.post(last[b:b + 1, :n].transpose(1, 2))[0, 0].numpy()
        r = rel_rms(wav[b, :n].cpu().numpy(), ref)
        worst["post"] = (max(worst.get("post", (0, 0))[0], r), 0.0)
        assert r <= STAGE_REL, ("post", b, r)
    for name, (r, edge) in worst.items():
        record(f"vocoder_{name}", rel_rms=r, edge_rel_rms=edge)


def test_vocoder_speaker_embedding_on_device(golden):
    voc, _ = _vocoder("tiny")
    spk = voc.speaker(torch.from_numpy(golden["tiny_bv_mel_ref"]).cuda())
    np.testing.assert_allclose(spk.cpu().numpy(), golden["tiny_bv_spk"], rtol=1e-3, atol=1e-3)


def test_vocoder_ragged_batch_equals_single():
    """Utterances of different lengths in one batch produce what each produces alone (bit-exact)."""
    voc, orc = _vocoder("tiny")
    torch.manual_seed(3)
    T = 11
    lat = torch.randn(3, T, 256)
    spk = torch.randn(3, 512)
    lens = torch.tensor([11, 6, 1])
    wav, _ = voc.forward(lat.cuda(), lens, spk.cuda(), want_pcm=False)
    for b in range(3):
        L = int(lens[b])
        w1, _ = voc.forward(lat[b:b + 1, :L].cuda(), torch.tensor([L]), spk[b:b + 1].cuda(), want_pcm=False)
        torch.testing.assert_close(wav[b, :L * 1024].cpu(), w1[0].cpu(), rtol=0, atol=0)
        ref = orc.forward(lat[b:b + 1, :L], spk[b:b + 1])[0, 0]
        rel = float(((w1[0].cpu() - ref) ** 2).mean().sqrt() / (ref ** 2).mean().sqrt())
        assert rel <= 2e-2, rel


@pytest.mark.parametrize("C,k,d,use_act,nres,alpha", [(24, 7, 3, True, 1, 1.0), (48, 11, 5, True, 2, 1.0 / 3),
                                                     (96, 3, 1, False, 0, 1.0), (24, 3, 1, True, 0, 1.0),
                                                     (96, 11, 5, True, 1, 1.0), (48, 7, 1, False, 2, 0.5),
                                                     # the product's conv-only forms (activation in its own kernel)
                                                     (24, 11, 5, False, 1, 1.0), (48, 11, 5, False, 1, 1.0),
                                                     (96, 7, 3, False, 2, 0.5)])
def test_amp_conv_matches_torch(C, k, d, use_act, nres, alpha):
    """itts_amp_conv_fwd = alpha * (conv(act(x)) + bias + r1 + r2) on a ragged batch vs torch fp32 with
    the torch-path Activation1d (oracle) rounded to bf16 as the kernel stages it.
    Tolerance: |err| <= 2e-2 * conv(|act|, |W|) + 1e-2 * |ref| (bf16 act staging and output)."""
    from indextts.utils.synthetic import kaiser_sinc_lowpass
    from indextts.vocoder.bigvgan import _Conv, conv1d_taps
    from oracle.bigvgan_oracle import activation1d
    _hip, lib = _lib()
    torch.manual_seed(C * k + d)
    B, T = 3, 300
    lens = torch.tensor([300, 57, 5], dtype=torch.int32)
    x = torch.randn(B, T, C).to(torch.bfloat16)
    res = [torch.randn(B, T, C).to(torch.bfloat16) for _ in range(nres)]
    w = torch.randn(C, C, k) / (C * k) ** 0.5
    bias = torch.randn(C) * 0.1
    filt = torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).reshape(-1)
    la, lb = torch.randn(C) * 0.3, torch.randn(C) * 0.3
    conv = _Conv(*conv1d_taps(w, d), bias, C, C, "cuda")
    xd, lensd = x.cuda(), lens.cuda()
    rd = [r.cuda() for r in res]
    fd, lad, lbd = filt.cuda(), la.cuda(), lb.cuda()
    y = torch.zeros(B, T, C, dtype=torch.bfloat16, device="cuda")
    _hip.check(lib.itts_amp_conv_fwd(
        xd.data_ptr(), T * C, C, fd.data_ptr() if use_act else None, fd.data_ptr() if use_act else None,
        lad.data_ptr() if use_act else None, lbd.data_ptr() if use_act else None, conv.w.data_ptr(),
        conv.bias.data_ptr(), rd[0].data_ptr() if nres > 0 else None, rd[1].data_ptr() if nres > 1 else None,
        y.data_ptr(), T * C, C, lensd.data_ptr(), B, T, C, C, conv.ntaps, conv.offs, alpha, _hip.stream_ptr()),
        "amp_conv")
    torch.cuda.synchronize()
    wq = w.to(torch.bfloat16).float()
    for b in range(B):
        L = int(lens[b])
        xb = x[b:b + 1, :L].float().transpose(1, 2)
        if use_act:
            xb = activation1d(xb, filt, filt, la, lb).to(torch.bfloat16).float()
        ref = F.conv1d(xb, wq, bias, dilation=d, padding=d * (k - 1) // 2)[0].t()
        for r in res:
            ref = ref + r[b, :L].float()
        ref = alpha * ref
        scale = alpha * F.conv1d(xb.abs(), wq.abs(), dilation=d, padding=d * (k - 1) // 2)[0].t()
        err = (y[b, :L].float().cpu() - ref).abs()
        assert bool((err <= 2e-2 * scale + 1e-2 * ref.abs() + 1e-3).all()), (b, float(err.max()))


@pytest.mark.parametrize("cin,k,d", [(192, 11, 5), (192, 3, 1), (384, 1, 1)])
def test_igemm_cout192_whole_width_tile_equals_64_column_tiles(monkeypatch, cin, k, d):
    """Cout = 192 (generator stage 2) on 256 x 192 tiles (default) is bit-identical to the 256 x 64
    tiles (ITTS_IG192=0): the same K-step order (channel chunk, tap) and MFMA blocks per output.
    bf16 output with both residuals and alpha, as the AMP layers call it; ragged lengths."""
    from indextts.vocoder.bigvgan import _Conv, conv1d_taps
    _hip, lib = _lib()
    torch.manual_seed(cin + k)
    B, T, cout = 3, 3000, 192
    lens = torch.tensor([3000, 1, 1234], dtype=torch.int32).cuda()
    x = torch.randn(B, T, cin).to(torch.bfloat16).cuda()
    r1, r2 = (torch.randn(B, T, cout).to(torch.bfloat16).cuda() for _ in range(2))
    conv = _Conv(*conv1d_taps(torch.randn(cout, cin, k) / (cin * k) ** 0.5, d), torch.randn(cout) * 0.1,
                 cin, cout, "cuda")
    outs = []
    for v in ("1", "0"):
        monkeypatch.setenv("ITTS_IG192", v)
        y = torch.full((B, T, cout), 3.0, dtype=torch.bfloat16, device="cuda")
        _hip.check(lib.itts_igemm_fwd(x.data_ptr(), T * cin, cin, conv.w.data_ptr(), conv.bias.data_ptr(), None,
                                      r1.data_ptr(), r2.data_ptr(), y.data_ptr(), T * cout, cout, lens.data_ptr(), B,
                                      T, cin, cout, conv.ntaps, conv.offs, 1, 0, 0.5, 0, _hip.BF16,
                                      _hip.stream_ptr()), "igemm")
        torch.cuda.synchronize()
        outs.append(y)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("ci,co,k,u", [(192, 96, 4, 4), (96, 48, 4, 2), (48, 24, 4, 2), (384, 192, 4, 4),
                                       (768, 384, 8, 4)])
def test_convtranspose_phases_as_output_columns_matches_torch(ci, co, k, u):
    """ConvTranspose1d(k, stride u, padding (k-u)/2) as ONE implicit GEMM with the u phases as output
    column blocks (convtr_fused): the [T][u*co] output read as [T*u][co] equals torch's
    conv_transpose1d on the bf16-rounded operands (f32 accumulation), per utterance of a ragged
    batch; output rows past len*u are not written.  Tolerance as test_igemm_conv_matches_torch."""
    from indextts.vocoder.bigvgan import _Conv, convtr_fused
    _hip, lib = _lib()
    torch.manual_seed(ci + k)
    B, T = 2, 300
    lens = torch.tensor([T, 77], dtype=torch.int32)
    x = torch.randn(B, T, ci).to(torch.bfloat16)
    w = torch.randn(ci, co, k) / (ci * k / u) ** 0.5
    bias = torch.randn(co) * 0.1
    taps, offs = convtr_fused(w, u, (k - u) // 2)
    conv = _Conv(taps, offs, bias.repeat(u), ci, u * co, "cuda")
    y = torch.full((B, T * u, co), 9.0, device="cuda")
    xd, lensd = x.cuda(), lens.cuda()
    _hip.check(lib.itts_igemm_fwd(xd.data_ptr(), T * ci, ci, conv.w.data_ptr(), conv.bias.data_ptr(), None, None,
                                  None, y.data_ptr(), T * u * co, u * co, lensd.data_ptr(), B, T, ci, u * co,
                                  conv.ntaps, conv.offs, 1, 0, 1.0, 0, _hip.F32, _hip.stream_ptr()), "igemm")
    torch.cuda.synchronize()
    wq = w.to(torch.bfloat16).float()
    for b in range(B):
        L = int(lens[b])
        xb = x[b:b + 1, :L].float().transpose(1, 2)
        ref = F.conv_transpose1d(xb, wq, bias, stride=u, padding=(k - u) // 2)[0].t()
        scale = F.conv_transpose1d(xb.abs(), wq.abs(), stride=u, padding=(k - u) // 2)[0].t()
        assert ref.shape[0] == L * u
        err = (y[b, :L * u].cpu() - ref).abs()
        assert bool((err <= 1e-4 * scale + 1e-5).all()), float(err.max())
        assert bool((y[b, L * u:] == 9.0).all())


@pytest.mark.parametrize("C,K", [(24, 7), (8, 3), (16, 15), (32, 7)])
def test_fused_tail_equals_activation_then_conv_post(C, K):
    """itts_act_conv_post_tanh (activation_post -> conv_post -> tanh -> int16 in one launch, round 6) is
    BIT-identical to itts_aa_snakebeta_fwd (bf16, MFMA path) followed by itts_conv_post_tanh on its bf16 output:
    wav and pcm, ragged lengths around the 448-sample job edges and the 32-sample activation tiles, utterances
    shorter than the activation's 3-sample edge zones (1, 2, 5, 6, 7 samples)."""
    from indextts.utils.synthetic import kaiser_sinc_lowpass
    _hip, lib = _lib()
    g = torch.Generator().manual_seed(C * 31 + K)
    T = 2000
    lens = torch.tensor([T, 1, 2, 5, 6, 7, 447, 448, 449, 896, 897, 31, 33, 1343, 1345, 1999], dtype=torch.int32)
    B = lens.numel()
    x = (torch.randn(B, T, C, generator=g) * 1.5).to(torch.bfloat16).cuda()
    up = torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).reshape(-1).float().cuda()
    down = (torch.from_numpy(kaiser_sinc_lowpass(0.25, 0.3, 12)).reshape(-1).float() * 1.01).cuda()
    la, lb = (torch.randn(C, generator=g) * 0.5).cuda(), (torch.randn(C, generator=g) * 0.5).cuda()
    w = (torch.randn(C, K, generator=g) / (C * K) ** 0.5).cuda()
    bias = 0.03
    ld = lens.cuda()
    s = _hip.stream_ptr()
    t1 = torch.zeros(B, T, C, dtype=torch.bfloat16, device="cuda")
    _hip.check(lib.itts_aa_snakebeta_fwd(x.data_ptr(), t1.data_ptr(), up.data_ptr(), down.data_ptr(), la.data_ptr(),
                                         lb.data_ptr(), ld.data_ptr(), B, C, T, T * C, C, 1, T * C, C, 1, _hip.BF16,
                                         _hip.BF16, s), "act")
    want_w = torch.full((B, T), 7.0, device="cuda")
    want_p = torch.full((B, T), 123, dtype=torch.int16, device="cuda")
    _hip.check(lib.itts_conv_post_tanh(t1.data_ptr(), T * C, C, w.data_ptr(), bias, C, K, ld.data_ptr(), B, T,
                                       want_w.data_ptr(), want_p.data_ptr(), T, _hip.BF16, s), "conv_post")
    got_w = torch.full((B, T), 7.0, device="cuda")
    got_p = torch.full((B, T), 123, dtype=torch.int16, device="cuda")
    _hip.check(lib.itts_act_conv_post_tanh(x.data_ptr(), T * C, C, up.data_ptr(), down.data_ptr(), la.data_ptr(),
                                           lb.data_ptr(), w.data_ptr(), bias, C, K, ld.data_ptr(), B, T,
                                           got_w.data_ptr(), got_p.data_ptr(), T, s), "fused tail")
    torch.cuda.synchronize()
    gw, ww = got_w.cpu(), want_w.cpu()
    bad = (gw.view(torch.int32) != ww.view(torch.int32)).nonzero()
    assert bad.numel() == 0, (bad[:8].tolist(), lens.tolist())
    assert torch.equal(got_p.cpu(), want_p.cpu())
    assert bool((gw[:, :] == 7.0).logical_or(torch.arange(T)[None] < lens[:, None]).all())  # nothing past len
