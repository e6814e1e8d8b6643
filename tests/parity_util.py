"""Shared parity checks for the GPU tests (test infrastructure, never imported by the product)."""
import numpy as np
import torch


def check_pcm(wav, pcm, ref_wav=None, ref_pcm=None):
    """The int16 output is EXACTLY trunc(clamp(32767 * wav, +-32767)) of the kernel's own f32
    waveform (quirk Q8; reference infer.py:627-631: ``torch.clamp(32767 * wav, -32767.0, 32767.0)``
    then ``.type(torch.int16)``).  Against a reference: |pcm - ref_pcm| <= ceil(32767 |wav - ref_wav|)
    + 1 element-wise, i.e. the int16 error is the float error, scaled, plus one truncation step."""
    w = torch.as_tensor(np.asarray(wav), dtype=torch.float32)
    want = torch.clamp(32767 * w, -32767.0, 32767.0).type(torch.int16)
    got = torch.as_tensor(np.asarray(pcm))
    assert got.dtype == torch.int16 and torch.equal(got, want), int((got.int() - want.int()).abs().max())
    if ref_pcm is not None:
        d = np.abs(np.asarray(pcm, np.int32) - np.asarray(ref_pcm, np.int32))
        bound = np.ceil(32767 * np.abs(np.asarray(wav, np.float64) - np.asarray(ref_wav, np.float64))) + 1
        assert (d <= bound).all(), int((d - bound).max())
