"""ECAPA-TDNN speaker embedding applied to the prompt mel inside every vocoder call.

Deterministic and per-prompt, so the host caches it (quirk Q6); PyTorch-ROCm code, not a
hand-written kernel target; convolutions as im2col GEMMs
(``utils/convgemm.py``, §8(f) item 2).

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


def _conv_same(x, sd, p, dilation=1, lin=None):
    w = sd[p + ".weight"]
    k = w.shape[-1]
    if lin is not None and k == 1 and x.shape[-1] > 1:  # 1x1 conv = linear layer over the time rows (bf16 MFMA)
        return lin(x.transpose(1, 2), p).transpose(1, 2)
    pad = dilation * (k - 1) // 2
    if pad > 0:
        x = F.pad(x, (pad, pad), mode="reflect")
    return conv1d(x, w, sd[p + ".bias"], dilation=dilation)


def _tdnn(x, sd, p, dilation=1, lin=None):
    return _bn(F.relu(_conv_same(x, sd, p + ".conv.conv", dilation, lin)), sd, p + ".norm.norm")


def _se_res2net(x, sd, p, dilation, scale=8, lin=None):
    residual = x
    h = _tdnn(x, sd, p + ".tdnn1", lin=lin)
    chunks = torch.chunk(h, scale, dim=1)
    ys = [chunks[0]]
    y = None
    for i in range(1, scale):
        inp = chunks[i] if i == 1 else chunks[i] + y
        y = _tdnn(inp, sd, f"{p}.res2net_block.blocks.{i - 1}", dilation)
        ys.append(y)
    h = _tdnn(torch.cat(ys, dim=1), sd, p + ".tdnn2", lin=lin)
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
    bf16 MFMA bank of the product mode for the 1x1 convolutions (utils/hiplinear.py; the reference
    runs BigVGAN under fp16 autocast, infer.py:613-623); None = f32 torch."""
    x = mel_ref.transpose(1, 2)
    x = _tdnn(x, sd, prefix + ".blocks.0")
    feats = []
    for i, dil in ((1, 2), (2, 3), (3, 4)):
        x = _se_res2net(x, sd, f"{prefix}.blocks.{i}", dil, lin=lin)
        feats.append(x)
    x = _tdnn(torch.cat(feats, dim=1), sd, prefix + ".mfa", lin=lin)
    L = x.shape[-1]
    uni = torch.full((1, 1, L), 1.0 / L, dtype=x.dtype, device=x.device)
    mean, std = _stats(x, uni)
    ctx = torch.cat([x, mean.unsqueeze(2).expand(-1, -1, L), std.unsqueeze(2).expand(-1, -1, L)], dim=1)
    a = torch.tanh(_tdnn(ctx, sd, prefix + ".asp.tdnn", lin=lin))
    a = torch.softmax(_conv_same(a, sd, prefix + ".asp.conv.conv"), dim=2)
    mean, std = _stats(x, a)
    pooled = torch.cat([mean, std], dim=1).unsqueeze(2)
    pooled = _bn(pooled, sd, prefix + ".asp_bn.norm")
    return _conv_same(pooled, sd, prefix + ".fc.conv").squeeze(2)
