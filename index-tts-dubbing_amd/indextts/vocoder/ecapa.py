"""ECAPA-TDNN speaker embedding applied to the prompt mel inside every vocoder call.

Deterministic and per-prompt, so the host caches it (quirk Q6).  Two numeric modes: the bf16 product
mode (``speaker_embedding_cl``) runs channel-last on the HIP kernels -- every conv on the MFMA implicit
GEMM over reflect-padded bf16 rows (``itts_pad_rows_bf16``), ReLU + BatchNorm as one affine kernel,
the pooling statistics in ``itts_time_stats`` (csrc/cond_ops.hip); the f32
verification mode (``speaker_embedding``) is f32 torch with the convolutions as im2col GEMMs
(``utils/convgemm.py``), the path the fp32 fixtures pin.

Reference behaviour followed:
  * ``ECAPA_TDNN.forward``                       BigVGAN/ECAPA_TDNN.py:543-581 (lengths=None)
  * ``TDNNBlock`` = BN(ReLU(conv))               BigVGAN/ECAPA_TDNN.py:96-101 region (forward)
  * speechbrain ``Conv1d`` "same" reflect pad: ``dil*(k-1)//2`` per side (the pad is derived from
    ``in_channels`` at nnet/CNN.py:480 but the difference L_in - L_out only depends on k and dil)
  * ``Res2NetBlock``: y0=x0, y1=f(x1), yi=f(xi + y_{i-1})
  * ``SEBlock`` (mean over time, 2 x 1x1 conv, sigmoid gate)
  * ``AttentiveStatisticsPooling`` (global context, eps 1e-12)  BigVGAN/ECAPA_TDNN.py:245-338
  * ``BatchNorm1d`` eval (running stats, eps 1e-5)             BigVGAN/nnet/normalization.py:13-108
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..utils.convgemm import conv1d


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.0, 1e-5)


def _conv_same(x, sd, p, dilation=1):
    w = sd[p + ".weight"]
    k = w.shape[-1]
    pad = dilation * (k - 1) // 2
    if pad > 0:
        x = F.pad(x, (pad, pad), mode="reflect")
    return conv1d(x, w, sd[p + ".bias"], dilation=dilation)


def _tdnn(x, sd, p, dilation=1):
    return _bn(F.relu(_conv_same(x, sd, p + ".conv.conv", dilation)), sd, p + ".norm.norm")


def _se_res2net(x, sd, p, dilation, scale=8):
    residual = x
    h = _tdnn(x, sd, p + ".tdnn1")
    chunks = torch.chunk(h, scale, dim=1)
    ys = [chunks[0]]
    y = None
    for i in range(1, scale):
        inp = chunks[i] if i == 1 else chunks[i] + y
        y = _tdnn(inp, sd, f"{p}.res2net_block.blocks.{i - 1}", dilation)
        ys.append(y)
    h = _tdnn(torch.cat(ys, dim=1), sd, p + ".tdnn2")
    s = h.mean(dim=2, keepdim=True)
    s = F.relu(_conv_same(s, sd, p + ".se_block.conv1.conv"))
    s = torch.sigmoid(_conv_same(s, sd, p + ".se_block.conv2.conv"))
    return s * h + residual


def _stats(x, w, eps=1e-12):
    mean = (w * x).sum(2)
    std = torch.sqrt((w * (x - mean.unsqueeze(2)).pow(2)).sum(2).clamp(eps))
    return mean, std


def speaker_embedding(sd, mel_ref, prefix="speaker_encoder", lin=None):
    """mel_ref [B, T, n_mels] -> [B, lin_neurons] (the reference returns [B, 1, lin]).  ``lin``: the
    bf16 MFMA ops of the product mode (utils/hiplinear.py; the reference runs BigVGAN under fp16
    autocast, infer.py:613-623) -> the channel-last path ``speaker_embedding_cl``; None = f32 torch."""
    if lin is not None:
        return speaker_embedding_cl(sd, mel_ref, lin, prefix)
    x = mel_ref.transpose(1, 2)
    x = _tdnn(x, sd, prefix + ".blocks.0")
    feats = []
    for i, dil in ((1, 2), (2, 3), (3, 4)):
        x = _se_res2net(x, sd, f"{prefix}.blocks.{i}", dil)
        feats.append(x)
    x = _tdnn(torch.cat(feats, dim=1), sd, prefix + ".mfa")
    L = x.shape[-1]
    uni = torch.full((1, 1, L), 1.0 / L, dtype=x.dtype, device=x.device)
    mean, std = _stats(x, uni)
    ctx = torch.cat([x, mean.unsqueeze(2).expand(-1, -1, L), std.unsqueeze(2).expand(-1, -1, L)], dim=1)
    a = torch.tanh(_tdnn(ctx, sd, prefix + ".asp.tdnn"))
    a = torch.softmax(_conv_same(a, sd, prefix + ".asp.conv.conv"), dim=2)
    mean, std = _stats(x, a)
    pooled = torch.cat([mean, std], dim=1).unsqueeze(2)
    pooled = _bn(pooled, sd, prefix + ".asp_bn.norm")
    return _conv_same(pooled, sd, prefix + ".fc.conv").squeeze(2)


# ---------------------------------------------------------------------------------------------------
# bf16 product path, channel-last [B, T, C] throughout (utils/hiplinear.HipLinearBank ops): every
# convolution on the MFMA igemm (k > 1 as taps over reflect-padded bf16 rows), ReLU + eval BatchNorm
# as one affine kernel, the Res2Net branches written into their slices of one buffer (no cat), and the
# attentive pooling's global-context concat folded into a per-row bias of its first 1x1 conv; the
# small per-utterance linears (SE, context, fc) on the same row-independent GEMM and the statistics
# over time in one kernel (itts_time_stats), so an utterance's embedding does not depend on its batch.  The reference's fp16 mode runs this module under autocast
# (infer.py:613-623).

def _se_res2net_cl(x, sd, p, dilation, ops, scale=8):
    B, T, C = x.shape
    h = ops.tdnn(x, p + ".tdnn1")
    w = C // scale
    cat = torch.empty_like(h)
    cat[..., :w] = h[..., :w]
    for i in range(1, scale):
        prev = None if i == 1 else cat[..., (i - 1) * w: i * w]
        ops.tdnn(h[..., i * w:(i + 1) * w], f"{p}.res2net_block.blocks.{i - 1}", dilation, x2=prev,
                 out=cat[..., i * w:(i + 1) * w])
    h = ops.tdnn(cat, p + ".tdnn2")
    s = F.relu(ops(ops.time_stats(h, want_std=False)[0], p + ".se_block.conv1.conv"))
    s = torch.sigmoid(ops(s, p + ".se_block.conv2.conv"))
    return torch.addcmul(x, h, s[:, None, :])


def speaker_embedding_cl(sd, mel_ref, ops, prefix="speaker_encoder"):
    """``speaker_embedding`` on the bf16 MFMA ops: mel_ref [B, T, n_mels] -> [B, lin_neurons]."""
    x = mel_ref.float().contiguous()
    x = ops.tdnn(x, prefix + ".blocks.0")
    feats = []
    for i, dil in ((1, 2), (2, 3), (3, 4)):
        x = _se_res2net_cl(x, sd, f"{prefix}.blocks.{i}", dil, ops)
        feats.append(x)
    x = ops.tdnn(torch.cat(feats, dim=-1), prefix + ".mfa")
    B, L, C = x.shape
    mean, std = ops.time_stats(x)
    # tdnn(cat([x, mean, std])) = W_x x + (W_m mean + W_s std + b): the context as a per-row bias
    q = prefix + ".asp.tdnn"
    key = q + ".conv.conv"
    if key + ".x.weight" not in ops.sd:
        wfull = sd[key + ".weight"][:, :, 0]
        ops.register(key + ".x", wfull[:, :C].contiguous(), None)
        ops.register(key + ".ctx", wfull[:, C:].contiguous(), sd[key + ".bias"])
    pb = ops(torch.cat([mean, std], -1), key + ".ctx")
    a = ops(x, key + ".x", bias=False) + pb[:, None, :]
    a = torch.tanh(ops.relu_bn(a, q + ".norm.norm"))
    # softmax over time and the weighted statistics in one row-independent kernel
    mean, std = ops.time_stats(x, ops(a, prefix + ".asp.conv.conv"))
    pooled = _bn(torch.cat([mean, std], dim=1).unsqueeze(2), sd, prefix + ".asp_bn.norm")[:, :, 0]
    return ops(pooled, prefix + ".fc.conv")
