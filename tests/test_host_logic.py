"""CPU tests of host-side logic: weight packing / polyphase decomposition against torch ops via an
emulation of the itts_igemm_fwd contract, config + synthetic weights, audio front-end."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from indextts.vocoder.bigvgan import conv1d_taps, convtr_phases, pack_dims_py, pack_taps


def igemm_emulate(x, taps, offs, T_out_rows, ymul=1, yoff=0, y=None):
    """Reference semantics of itts_igemm_fwd for one utterance: y[q*ymul+yoff] = sum_j W_j x[q+off_j]."""
    T, Cin = x.shape
    Cout = taps[0].shape[0]
    if y is None:
        y = torch.zeros(T_out_rows, Cout)
    for q in range(T):
        acc = torch.zeros(Cout)
        for w, o in zip(taps, offs):
            t = q + o
            if 0 <= t < T:
                acc += w @ x[t]
        y[q * ymul + yoff] = acc
    return y


@pytest.mark.parametrize("k,d", [(3, 1), (3, 5), (7, 3), (11, 5), (7, 1)])
def test_conv1d_taps(k, d):
    torch.manual_seed(0)
    x = torch.randn(1, 6, 40)
    w = torch.randn(5, 6, k)
    ref = F.conv1d(x, w, dilation=d, padding=d * (k - 1) // 2)[0].t()
    taps, offs = conv1d_taps(w, d)
    got = igemm_emulate(x[0].t(), taps, offs, 40)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("u,K", [(4, 8), (4, 4), (2, 4)])
def test_convtranspose_polyphase(u, K):
    torch.manual_seed(1)
    L = 13
    x = torch.randn(1, 6, L)
    w = torch.randn(6, 5, K)
    P = (K - u) // 2
    ref = F.conv_transpose1d(x, w, stride=u, padding=P)[0].t()
    assert ref.shape[0] == u * L
    y = torch.zeros(u * L, 5)
    for rho, (taps, offs) in enumerate(convtr_phases(w, u, P)):
        igemm_emulate(x[0].t(), taps, offs, u * L, ymul=u, yoff=rho, y=y)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)


def test_pack_layout():
    w = [torch.randn(40, 24), torch.randn(40, 24)]
    p = pack_taps(w, 24, 40)
    ci, co = pack_dims_py(24, 40)
    assert p.shape == (2, co, ci) and p.dtype == torch.bfloat16
    assert torch.equal(p[1, :40, :24].float(), w[1].to(torch.bfloat16).float())
    assert float(p[:, 40:].abs().sum()) == 0 and float(p[:, :, 24:].abs().sum()) == 0


def test_mel_front_end_matches_numpy_restatement():
    """MelSpectrogramFeatures (CPU restatement of torchaudio MelSpectrogram + safe_log; parity unpinned:
    torchaudio is absent) vs a from-spec numpy version (reflect pad, periodic Hann, rfft, HTK mels)."""
    import numpy as np
    import torch
    from indextts.utils.audio import MelSpectrogramFeatures, mel_filterbank
    g = np.random.default_rng(0)
    x = (0.3 * g.standard_normal(24000 // 2)).astype(np.float32)
    got = MelSpectrogramFeatures()(torch.from_numpy(x)[None])[0].numpy()
    n_fft, hop = 1024, 256
    xp = np.pad(x.astype(np.float64), (n_fft // 2, n_fft // 2), mode="reflect")
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    frames = np.stack([xp[i * hop: i * hop + n_fft] * win for i in range(len(x) // hop + 1)])
    mag = np.abs(np.fft.rfft(frames, axis=1))
    fb = mel_filterbank(n_fft // 2 + 1, 0.0, 12000.0, 100, 24000).double().numpy()
    want = np.log(np.maximum(mag @ fb, 1e-7)).T
    assert got.shape == want.shape
    np.testing.assert_allclose(np.exp(got), np.exp(want), rtol=1e-4, atol=1e-5)
