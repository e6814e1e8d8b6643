"""Deterministic 1-D / 2-D convolutions as GEMMs for the per-prompt modules (conditioning encoder,
ECAPA speaker encoder).

MIOpen's only deterministic algorithm for these small fp32 convolutions is its naive direct kernel
(``naive_conv_ab_nonpacked_fwd_nchw_float``: 8.6 ms per batch of 32 prompts in round 1).  Here every
convolution is an explicit im2col view (``Tensor.unfold``, no copy until the GEMM needs it) times the
weight matrix on hipBLASLt -- a fixed reduction order for fixed shapes, so the prompt features stay
run-to-run identical (tests/test_gpu_pipeline.py) -- and the depthwise k=15 conformer convolution is
an unfolded multiply-sum.  fp32 throughout, same math as ``F.conv1d`` / ``F.conv2d``.

Reference ops replaced: ``ConvolutionModule`` pointwise/depthwise convs
(gpt/conformer_encoder.py:108-167), ``Conv2dSubsampling2`` (gpt/conformer/subsampling.py:164-190),
speechbrain ``Conv1d`` in ``TDNNBlock`` / ``SEBlock`` / ASP (BigVGAN/ECAPA_TDNN.py, nnet/CNN.py:411-488).
"""
from __future__ import annotations

from typing import Optional

import torch


def conv1d(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None, dilation: int = 1,
           padding: int = 0, groups: int = 1) -> torch.Tensor:
    """``F.conv1d(x, w, b, stride=1, padding=padding, dilation=dilation, groups=groups)`` for
    groups == 1 or depthwise (groups == C_in == C_out).  x [B, C_in, T] -> [B, C_out, T_out]."""
    if padding:
        x = torch.nn.functional.pad(x, (padding, padding))
    B, Cin, T = x.shape
    Cout, Cg, k = w.shape
    span = dilation * (k - 1) + 1
    if groups == 1:
        assert Cg == Cin, (w.shape, x.shape)
        if k == 1:
            y = torch.matmul(w[:, :, 0], x)  # [Cout, Cin] @ [B, Cin, T]
        else:
            cols = x.unfold(2, span, 1)[..., ::dilation]  # [B, Cin, T_out, k]
            T_out = cols.shape[2]
            cols = cols.permute(0, 2, 1, 3).reshape(B, T_out, Cin * k)
            y = torch.matmul(cols, w.reshape(Cout, Cin * k).t()).transpose(1, 2)
    else:
        assert groups == Cin == Cout and Cg == 1, "only full or depthwise convolutions"
        cols = x.unfold(2, span, 1)[..., ::dilation]  # [B, C, T_out, k]
        y = (cols * w[:, 0][None, :, None, :]).sum(-1)
    if b is not None:
        y = y + b[None, :, None]
    return y.contiguous()


def conv2d_s2(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.conv2d(x, w, b, stride=2)`` (no padding).  x [B, C_in, H, W] -> [B, C_out, H', W']."""
    B, Cin, H, W = x.shape
    Cout, _, kh, kw = w.shape
    cols = x.unfold(2, kh, 2).unfold(3, kw, 2)  # [B, Cin, H', W', kh, kw]
    Ho, Wo = cols.shape[2], cols.shape[3]
    cols = cols.permute(0, 2, 3, 1, 4, 5).reshape(B, Ho * Wo, Cin * kh * kw)
    y = torch.matmul(cols, w.reshape(Cout, -1).t())  # [B, H'W', Cout]
    if b is not None:
        y = y + b
    return y.transpose(1, 2).reshape(B, Cout, Ho, Wo).contiguous()
