"""Prompt audio front-end: wav I/O, sinc resampling and the log-mel features.

The reference uses torchaudio (``torchaudio.load`` / ``transforms.Resample`` /
``transforms.MelSpectrogram``; ``indextts/infer.py:509-514``,
``indextts/utils/feature_extractors.py:24-50``).  torchaudio is not in this image, so this module
restates those published algorithms on plain torch ops:

  * load: 16-bit PCM -> float32 in [-1, 1) (x / 32768), channels first
  * resample: torchaudio's ``sinc_interp_hann`` kernel (lowpass_filter_width 6, rolloff 0.99)
  * mel: |STFT| (n_fft 1024, hop 256, periodic Hann, center + reflect pad, power 1) @ HTK
    triangular filterbank (f_min 0, f_max sr/2, no norm), then ``safe_log`` clip 1e-7
    (``indextts/utils/common.py:110-121``)

torchaudio being absent, these are *parity unpinned* against the reference's own front-end
(SURVEY.md §8(f) item 1); they are tested against from-spec numpy restatements instead.
"""
from __future__ import annotations

import math
import wave

import numpy as np
import torch
import torch.nn.functional as F


def load_wav(path: str):
    """-> (float32 tensor [channels, frames], sample_rate). 16-bit (and 8/32-bit) PCM wav."""
    with wave.open(path, "rb") as w:
        ch, sw, sr, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if sw == 2:
        a = np.frombuffer(raw, dtype="<i2").astype(np.float32) / 32768.0
    elif sw == 4:
        a = np.frombuffer(raw, dtype="<i4").astype(np.float32) / 2147483648.0
    elif sw == 1:
        a = (np.frombuffer(raw, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"unsupported sample width {sw} in {path}")
    return torch.from_numpy(a.reshape(-1, ch).T.copy()), sr


def save_wav_int16(path: str, pcm: np.ndarray, sr: int):
    """pcm: int16 [frames] or [frames, channels] (the reference writes via torchaudio.save)."""
    pcm = np.asarray(pcm, dtype=np.int16)
    if pcm.ndim == 1:
        pcm = pcm[:, None]
    with wave.open(path, "wb") as w:
        w.setnchannels(pcm.shape[1])
        w.setsampwidth(2)
        w.setframerate(int(sr))
        w.writeframes(pcm.astype("<i2").tobytes())


def sinc_resample_kernel(orig: int, new: int, width_zc: int = 6, rolloff: float = 0.99):
    g = math.gcd(orig, new)
    orig, new = orig // g, new // g
    base = min(orig, new) * rolloff
    width = math.ceil(width_zc * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=torch.float64)[:, None, None] / new + idx
    t = (t * base).clamp(-width_zc, width_zc)
    win = torch.cos(t * math.pi / width_zc / 2) ** 2
    t = t * math.pi
    k = torch.where(t == 0, torch.ones_like(t), torch.sin(t) / t) * win * (base / orig)
    return k, orig, new, width


def resample(wav: torch.Tensor, orig_sr: int, new_sr: int) -> torch.Tensor:
    """wav [..., L] float32 -> [..., ceil(new*L/orig)]."""
    if orig_sr == new_sr:
        return wav
    k, o, n, width = sinc_resample_kernel(orig_sr, new_sr)
    shape = wav.shape
    x = wav.reshape(-1, 1, shape[-1])
    x = F.pad(x, (width, width + o))
    y = F.conv1d(x, k.to(wav.device, wav.dtype), stride=o)  # [N, new, frames]
    y = y.transpose(1, 2).reshape(x.shape[0], -1)
    target = math.ceil(n * shape[-1] / o)
    return y[..., :target].reshape(*shape[:-1], -1)


def resample_hip(wav: torch.Tensor, orig_sr: int, new_sr: int) -> torch.Tensor:
    """``resample`` on the GPU (itts_resample_sinc, csrc/frontend.hip): wav [..., L] f32 on a HIP device."""
    from .. import _hip
    if orig_sr == new_sr:
        return wav
    k, o, n, width = sinc_resample_kernel(orig_sr, new_sr)
    shape = wav.shape
    x = wav.reshape(-1, shape[-1]).float().contiguous()
    B, L = x.shape
    target = math.ceil(n * L / o)
    kern = k.reshape(n, -1).to(wav.device, torch.float32).contiguous()
    y = torch.empty(B, target, dtype=torch.float32, device=wav.device)
    lib = _hip.load()
    _hip.check(lib.itts_resample_sinc(x.data_ptr(), x.stride(0), B, L, kern.data_ptr(), o, n, width, y.data_ptr(),
                                      y.stride(0), target, _hip.stream_ptr(wav.device)), "itts_resample_sinc")
    return y.reshape(*shape[:-1], target)


def mel_filterbank(n_freqs: int, f_min: float, f_max: float, n_mels: int, sr: int) -> torch.Tensor:
    """HTK triangular filterbank [n_freqs, n_mels] (no area normalisation)."""
    all_f = torch.linspace(0, sr // 2, n_freqs)
    hz2mel = lambda f: 2595.0 * math.log10(1.0 + f / 700.0)
    m = torch.linspace(hz2mel(f_min), hz2mel(f_max), n_mels + 2)
    f_pts = 700.0 * (10 ** (m / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_f[:, None]
    down = -slopes[:, :-2] / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.clamp(torch.minimum(down, up), min=0.0)


class MelSpectrogramFeatures:
    """``MelSpectrogramFeatures()(audio) -> log-mel [B, 100, frames]`` (center padding)."""

    def __init__(self, sample_rate=24000, n_fft=1024, hop_length=256, win_length=None, n_mels=100,
                 mel_fmin=0, mel_fmax=None, normalize=False, padding="center"):
        if padding not in ("center", "same"):
            raise ValueError("Padding must be 'center' or 'same'.")
        self.sr, self.n_fft, self.hop = sample_rate, n_fft, hop_length
        self.win = win_length or n_fft
        self.padding = padding
        self.fb = mel_filterbank(n_fft // 2 + 1, float(mel_fmin), float(mel_fmax or sample_rate / 2), n_mels,
                                 sample_rate)

    def __call__(self, audio: torch.Tensor) -> torch.Tensor:
        if self.padding == "same":
            pad = self.win - self.hop
            audio = F.pad(audio, (pad // 2, pad // 2), mode="reflect")
        shape = audio.shape
        x = audio.reshape(-1, shape[-1])
        window = torch.hann_window(self.win, periodic=True, dtype=x.dtype, device=x.device)
        spec = torch.stft(x, self.n_fft, self.hop, self.win, window, center=(self.padding == "center"),
                          pad_mode="reflect", normalized=False, onesided=True, return_complex=True).abs()
        mel = (spec.transpose(-1, -2) @ self.fb.to(x.device, x.dtype)).transpose(-1, -2)
        mel = mel.reshape(*shape[:-1], mel.shape[-2], mel.shape[-1])
        return torch.log(torch.clamp(mel, min=1e-7))


def log_mel_hip(audio: torch.Tensor, feats: "MelSpectrogramFeatures" = None) -> torch.Tensor:
    """``MelSpectrogramFeatures()(audio)`` (center padding) on the GPU: audio [B, L] f32 on a HIP
    device -> [B, n_mels, L // hop + 1] via the fused itts_log_mel kernel (csrc/frontend.hip)."""
    from .. import _hip
    feats = feats or MelSpectrogramFeatures()
    assert feats.padding == "center" and feats.win == feats.n_fft, "HIP log-mel implements the center/full-window form"
    lib = _hip.load()
    x = audio.reshape(-1, audio.shape[-1]).float().contiguous()
    B, L = x.shape
    dev = x.device
    window = torch.hann_window(feats.win, periodic=True, dtype=torch.float32, device=dev)
    fb = feats.fb.to(dev, torch.float32).contiguous()
    out = torch.empty(B, fb.shape[1], L // feats.hop + 1, device=dev)
    _hip.check(lib.itts_log_mel(x.data_ptr(), x.stride(0), B, L, window.data_ptr(), fb.data_ptr(), feats.n_fft,
                                feats.hop, fb.shape[1], out.data_ptr(), _hip.stream_ptr(dev)), "itts_log_mel")
    return out.reshape(*audio.shape[:-1], out.shape[-2], out.shape[-1])


def prompt_mel(path: str, device=None) -> torch.Tensor:
    """The prompt-mel pipeline of ``infer()`` (``indextts/infer.py:509-514``) -> [1, 100, frames].
    ``device`` (a HIP device): resampling and the log-mel run there on the HIP kernels
    (itts_resample_sinc, itts_log_mel);
    None: the CPU restatement (used by the tests as the from-spec reference)."""
    audio, sr = load_wav(path)
    audio = torch.mean(audio, dim=0, keepdim=True)
    if device is not None and torch.device(device).type == "cuda":
        audio = audio.to(device)
        return log_mel_hip(resample_hip(audio, sr, 24000))
    audio = resample(audio, sr, 24000)
    return MelSpectrogramFeatures()(audio)
