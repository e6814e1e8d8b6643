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


def bf16_effective_gpt_sds(sd, n_layer, rounding=True):
    """The GPT weights as the bf16 product path stores them, as two f32 state dicts for
    ``GPTOracle(sd_prefill, cfg, sd_decode=...)``, so that an oracle run on them differs from the GPU only by
    activation rounding and summation order:

      * prefill / latent GEMMs (itts_igemm_fwd over ``pack_taps``): bf16(W) of c_attn / attn.c_proj / mlp.c_fc /
        mlp.c_proj, LayerNorms as they are;
      * decode steps (itts_decode_gemm16x / the persistent layer, engine.fold_ln_weights -> itts_gpt_fold_ln,
        gpt_pack.hip:32-56): ln_1 / ln_2 folded into c_attn / c_fc -- W' = bf16(f32(diag(g) W)) and the bias
        c = b^T W + bias (double sums), applied behind an affine-free LayerNorm (rstd (x W' - mu 1^T W') + c is
        LN(x) W' + c exactly) -- attn.c_proj / mlp.c_proj bf16(W);
      * mel_head bf16(W) in both; embeddings, biases, ln_f / final_norm f32 (they are f32 on the device).
    ``rounding=False``: the same folding without the bf16 rounding (a CPU test checks the fold is exact).
    """
    base = {k: torch.as_tensor(np.asarray(v)).float().clone() for k, v in sd.items()}
    r16 = (lambda t: t.float().to(torch.bfloat16).float()) if rounding else (lambda t: t.float())  # noqa: E731
    pre, dec = dict(base), dict(base)
    for i in range(n_layer):
        p = f"gpt.h.{i}"
        for k in ("attn.c_attn", "attn.c_proj", "mlp.c_fc", "mlp.c_proj"):
            pre[f"{p}.{k}.weight"] = r16(base[f"{p}.{k}.weight"])
        for ln, k in (("ln_1", "attn.c_attn"), ("ln_2", "mlp.c_fc")):
            g, b = base[f"{p}.{ln}.weight"].double(), base[f"{p}.{ln}.bias"].double()
            w = base[f"{p}.{k}.weight"].double()  # HF Conv1D [in, out]
            dec[f"{p}.{k}.weight"] = r16((w * g[:, None]).float())
            dec[f"{p}.{k}.bias"] = (b @ w + base[f"{p}.{k}.bias"].double()).float()
            dec[f"{p}.{ln}.weight"] = torch.ones_like(base[f"{p}.{ln}.weight"])
            dec[f"{p}.{ln}.bias"] = torch.zeros_like(base[f"{p}.{ln}.bias"])
        for k in ("attn.c_proj", "mlp.c_proj"):
            dec[f"{p}.{k}.weight"] = r16(base[f"{p}.{k}.weight"])
    pre["mel_head.weight"] = dec["mel_head.weight"] = r16(base["mel_head.weight"])
    return pre, dec
