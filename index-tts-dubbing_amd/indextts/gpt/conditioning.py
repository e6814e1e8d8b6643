"""Speech-prompt conditioning: conformer encoder + perceiver resampler -> ``conds [B, 32, D]``.

Runs once per prompt (cached by the caller, quirk Q6).  With a ``lin`` bank (bf16 product mode,
``utils/hiplinear.py``) every linear / pointwise conv runs on the HIP MFMA implicit GEMM and the
subsampling conv, rel-pos attention, GLU / depthwise / LayerNorm / SiLU run as HIP kernels
(csrc/cond_ops.hip); without it (f32 verification mode) it is f32 torch with
the convolutions as explicit im2col GEMMs (``utils/convgemm.py``: deterministic without MIOpen's naive
direct kernel).  Functional restatement over the reference state-dict.

Reference behaviour followed (file:line in the reference tree):
  * ``UnifiedVoice.get_conditioning`` conformer_perceiver branch  gpt/model.py:496-502
  * ``BaseEncoder.forward``                                          gpt/conformer_encoder.py:400-436
  * ``Conv2dSubsampling2.forward`` (mask ``[:, :, 2::2]``)           gpt/conformer/subsampling.py:164-190
  * ``RelPositionalEncoding.forward`` (x*sqrt(C); pe[:, :T])        gpt/conformer/embedding.py:127-142
  * ``ConformerEncoderLayer.forward`` (pre-LN, no macaron)          gpt/conformer_encoder.py:247-313
  * ``RelPositionMultiHeadedAttention.forward`` (no rel_shift)       gpt/conformer/attention.py:235-312
  * ``ConvolutionModule.forward`` (GLU, depthwise k15, LN, SiLU)     gpt/conformer_encoder.py:108-167
  * ``PerceiverResampler.forward`` / ``Attention`` / ``Attend``       gpt/perceiver.py:263-274, 296-317, 111-150
  * ``RMSNorm`` (F.normalize * sqrt(D) * gamma)                     gpt/perceiver.py:167-186
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ..utils.convgemm import conv1d, conv2d_s2


def _lin(x, sd, name, bias=True, lin=None):
    """F.linear in f32, or ``lin(x, name, bias)``: the bf16 MFMA bank of the product mode
    (utils/hiplinear.py; the reference computes these under fp16 autocast, infer.py:572-586)."""
    if lin is not None:
        return lin(x, name, bias)
    return F.linear(x, sd[name + ".weight"], sd.get(name + ".bias") if bias else None)


def _ln(x, sd, name, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[name + ".weight"], sd[name + ".bias"], eps)


def _rel_pos_mha(x, sd, p, heads, mask, pos_emb, lin=None):
    if lin is not None:  # fused qkv GEMM + HIP attention (csrc/cond_ops.hip), bf16 into linear_out
        return lin.rel_attn(x, p, heads, mask, pos_emb)
    B, T, C = x.shape
    dk = C // heads
    q = _lin(x, sd, p + ".linear_q", lin=lin).view(B, T, heads, dk)
    k = _lin(x, sd, p + ".linear_k", lin=lin).view(B, T, heads, dk).transpose(1, 2)
    v = _lin(x, sd, p + ".linear_v", lin=lin).view(B, T, heads, dk).transpose(1, 2)
    pos = F.linear(pos_emb, sd[p + ".linear_pos.weight"]).view(pos_emb.shape[0], -1, heads, dk).transpose(1, 2)
    qu = (q + sd[p + ".pos_bias_u"]).transpose(1, 2)
    qv = (q + sd[p + ".pos_bias_v"]).transpose(1, 2)
    scores = (qu @ k.transpose(-2, -1) + qv @ pos.transpose(-2, -1)) / math.sqrt(dk)
    masked = ~mask.unsqueeze(1)  # [B, 1, 1, T]
    scores = scores.masked_fill(masked, float("-inf"))
    attn = torch.softmax(scores, dim=-1).masked_fill(masked, 0.0)
    out = (attn @ v).transpose(1, 2).reshape(B, T, C)
    return _lin(out, sd, p + ".linear_out", lin=lin)


def _conv_module(x, sd, p, mask, lin=None, residual=None):
    """residual (fast path, all frames valid): pointwise_conv2 adds into it in place, returns None."""
    C = x.shape[-1]
    if lin is not None:  # channel-last: the pointwise convs are linear layers over the rows
        h = x if residual is not None else x.masked_fill(~mask.transpose(1, 2), 0.0)
        h = lin.glu_dwconv(lin(h, p + ".pointwise_conv1"), p)  # GLU, depthwise, LN, SiLU fused (bf16 out)
        if residual is not None:
            lin(h, p + ".pointwise_conv2", out=residual, residual=residual)
            return None
        return lin(h, p + ".pointwise_conv2").masked_fill(~mask.transpose(1, 2), 0.0)
    h = x.transpose(1, 2).masked_fill(~mask, 0.0)  # [B, C, T]
    h = conv1d(h, sd[p + ".pointwise_conv1.weight"], sd[p + ".pointwise_conv1.bias"])
    h = F.glu(h, dim=1)
    w = sd[p + ".depthwise_conv.weight"]
    h = conv1d(h, w, sd[p + ".depthwise_conv.bias"], padding=(w.shape[-1] - 1) // 2, groups=C)
    h = F.silu(_ln(h.transpose(1, 2), sd, p + ".norm")).transpose(1, 2)
    h = conv1d(h, sd[p + ".pointwise_conv2.weight"], sd[p + ".pointwise_conv2.bias"])
    return h.masked_fill(~mask, 0.0).transpose(1, 2)


def conformer_encode(sd, mel, mel_lengths, heads: int, num_blocks: int, prefix="conditioning_encoder", lin=None,
                     full=False):
    """mel [B, n_mels, T] -> (xs [B, T', C], mask [B, 1, T']).  full: every frame valid (host-known)."""
    x = mel.transpose(1, 2)
    B, T, _ = x.shape
    valid = torch.arange(T, device=x.device)[None, :] < mel_lengths.to(x.device)[:, None]
    mask = valid.unsqueeze(1)
    p = prefix + ".embed"
    if lin is not None:  # fused conv + ReLU -> channel-last bf16, Linear on permuted columns
        h = lin.subsample_linear(lin.subsample(mel, p), p, sd[p + ".conv.0.weight"].shape[0])
        t = h.shape[1]
    else:
        h = F.relu(conv2d_s2(x.unsqueeze(1), sd[p + ".conv.0.weight"], sd[p + ".conv.0.bias"]))
        b, c, t, f = h.shape
        h = _lin(h.transpose(1, 2).reshape(b, t, c * f), sd, p + ".out.0", lin=lin)
    C = h.shape[-1]
    h = h * math.sqrt(C)
    pos_emb = sd[p + ".pos_enc.pe"][:, :t]
    mask = mask[:, :, 2::2]
    for i in range(num_blocks):
        q = f"{prefix}.encoders.{i}"
        if lin is not None:  # LN -> bf16 operands, residual adds and SiLU in the GEMM epilogues
            lin.rel_attn(lin.ln(h, q + ".norm_mha"), q + ".self_attn", heads, mask, pos_emb, residual=h)
            c = _conv_module(lin.ln(h, q + ".norm_conv"), sd, q + ".conv_module", mask, lin, residual=h if full else None)
            if c is not None:
                h = h + c
            f = lin(lin.ln(h, q + ".norm_ff"), q + ".feed_forward.w_1", act=2, bf16_out=True)
            lin(f, q + ".feed_forward.w_2", out=h, residual=h)
            h = _ln(h, sd, q + ".norm_final")
            continue
        h = h + _rel_pos_mha(_ln(h, sd, q + ".norm_mha"), sd, q + ".self_attn", heads, mask, pos_emb, lin)
        h = h + _conv_module(_ln(h, sd, q + ".norm_conv"), sd, q + ".conv_module", mask, lin)
        y = _ln(h, sd, q + ".norm_ff")
        h = h + _lin(F.silu(_lin(y, sd, q + ".feed_forward.w_1", lin=lin)), sd, q + ".feed_forward.w_2", lin=lin)
        h = _ln(h, sd, q + ".norm_final")
    return _ln(h, sd, prefix + ".after_norm"), mask


def perceiver_resample(sd, ctx, key_mask, heads: int, prefix="perceiver_encoder", lin=None):
    """ctx [B, T', C] + key_mask [B, 32 + T'] (True = keep) -> conds [B, 32, D]."""
    x = _lin(ctx, sd, prefix + ".proj_context", lin=lin)
    lat0 = sd[prefix + ".latents"]
    lat = lat0.unsqueeze(0).expand(x.shape[0], -1, -1)
    D = lat.shape[-1]
    neg = -torch.finfo(x.dtype).max
    for i in range(2):
        a = f"{prefix}.layers.{i}.0"
        context = torch.cat([lat, x], dim=1)
        q = _lin(lat, sd, a + ".to_q", bias=False, lin=lin)
        kv = _lin(context, sd, a + ".to_kv", bias=False, lin=lin)
        B, n, inner = q.shape
        dh = inner // heads
        if lin is not None:  # product mode: the HIP cross-attention kernel (row-independent, f32)
            out = lin.cross_attn(q, kv, key_mask, heads, dh ** -0.5)
        else:
            k, v = kv.chunk(2, dim=-1)
            q = q.view(B, n, heads, dh).transpose(1, 2)
            k = k.view(B, -1, heads, dh).transpose(1, 2)
            v = v.view(B, -1, heads, dh).transpose(1, 2)
            sim = (q @ k.transpose(-2, -1)) * (dh ** -0.5)
            sim = sim.masked_fill(~key_mask[:, None, None, :], neg)
            out = (sim.softmax(dim=-1) @ v).transpose(1, 2).reshape(B, n, inner)
        lat = _lin(out, sd, a + ".to_out", bias=False, lin=lin) + lat
        f = f"{prefix}.layers.{i}.1"
        hx, gate = _lin(lat, sd, f + ".0", lin=lin).chunk(2, dim=-1)
        lat = _lin(F.gelu(gate) * hx, sd, f + ".2", lin=lin) + lat
    return F.normalize(lat, dim=-1) * math.sqrt(D) * sd[prefix + ".norm.gamma"]


def get_conditioning(sd, cfg_gpt, mel, mel_lengths=None, lin=None):
    """``UnifiedVoice.get_conditioning`` for condition_type conformer_perceiver.

    mel [B, 100, T] float32 -> conds [B, 32, model_dim].  ``lin``: the bf16 MFMA linear bank of the
    product mode (utils/hiplinear.HipLinearBank); None = f32 torch (verification mode, oracle tests)."""
    if mel.ndim == 2:
        mel = mel.unsqueeze(0)
    full = mel_lengths is None  # every frame valid: known on the host (no mask work, fused residuals)
    if mel_lengths is None:
        mel_lengths = torch.full((mel.shape[0],), mel.shape[-1], dtype=torch.long, device=mel.device)
    cm = cfg_gpt.condition_module
    xs, mask = conformer_encode(sd, mel, mel_lengths, int(cm.attention_heads), int(cm.num_blocks), lin=lin,
                                full=full)
    key_mask = F.pad(mask.squeeze(1), (32, 0), value=True)
    return perceiver_resample(sd, xs, key_mask, int(cm.attention_heads), lin=lin)
