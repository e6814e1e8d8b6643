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


# ---- measured parity record -----------------------------------------------------------------------
# Every GPU parity test records the errors it measured (not just pass / fail) into
# gpurun_out/parity_<ITTS_PARITY_TAG>.json, merged key by key and rewritten after every record, so a
# `pytest -q` run leaves the numbers the bounds are set from (set each bound at <= 1.5x
# the measured value); the round's copy is committed as profiles/parity_rNN.json.
_RECORD = {}


def record(key, **values):
    import json
    import os
    clean = {}
    for k, v in values.items():
        if isinstance(v, (np.floating, np.integer)):
            v = v.item()
        elif isinstance(v, torch.Tensor):
            v = v.item()
        clean[k] = v
    _RECORD.setdefault(key, {}).update(clean)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "gpurun_out", f"parity_{os.environ.get('ITTS_PARITY_TAG', 'latest')}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    old = {}
    if os.path.exists(out):
        try:
            with open(out) as f:
                old = json.load(f)
        except (OSError, ValueError):
            old = {}
    old.update(_RECORD)
    with open(out + ".tmp", "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)
    os.replace(out + ".tmp", out)


def rel_rms(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return float(np.sqrt(np.mean((got - ref) ** 2) / np.mean(ref ** 2)))
