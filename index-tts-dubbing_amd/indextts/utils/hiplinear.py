"""Linear layers of the per-prompt modules on the MFMA implicit GEMM (bf16 operands, f32 accumulate).

The conditioning encoder + perceiver (``UnifiedVoice.get_conditioning``, gpt/model.py:496-502) and the
ECAPA speaker encoder (BigVGAN/ECAPA_TDNN.py:543-581) run, in the reference's fp16 product mode, under
``torch.amp.autocast`` (indextts/infer.py:572-586, 613-623): their GEMMs and convolutions compute in
half precision there.  The bf16 product mode here does the same with its own kernel:
``itts_igemm_fwd`` (csrc/igemm.hip) as a 1-tap GEMM -- inputs rounded to bf16, f32 accumulation and
f32 outputs, row-independent tiles (a prompt's features do not depend on the batch it shares).  The
exact-f32 verification mode keeps the f32 torch path (``linear=None``).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .. import _hip


class HipLinearBank:
    """``bank(x, name)`` = ``F.linear(x, sd[name + ".weight"], sd[name + ".bias"])`` (bias optional)
    for x [..., K] f32 or bf16; weights packed to bf16 on first use; 1x1 convolutions ([N, K, 1]
    weights) are linear layers over channel-last rows.  Also the conditioning encoder's two fused
    kernels (csrc/cond_ops.hip): ``subsample`` (Conv2dSubsampling2 -> channel-last bf16) and
    ``glu_dwconv`` (GLU + depthwise conv + LayerNorm + SiLU -> bf16)."""

    def __init__(self, sd: Dict[str, torch.Tensor], device):
        self.sd = sd
        self.dev = torch.device(device)
        self.lib = _hip.load()
        self._packed: Dict[object, tuple] = {}
        self.tiled = True  # LDS-tiled GLU/depthwise kernel where C allows (False: one step per workgroup)

    def register(self, name: str, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> None:
        """a derived weight (e.g. column-permuted) under its own name"""
        self.sd[name + ".weight"] = weight
        if bias is not None:
            self.sd[name + ".bias"] = bias

    def _pack(self, name: str):
        ent = self._packed.get(name)
        if ent is None:
            from ..vocoder.bigvgan import pack_taps
            w = self.sd[name + ".weight"].float()
            if w.ndim == 3:
                assert w.shape[-1] == 1, "only 1x1 convolutions are linear layers"
                w = w[:, :, 0]
            N, K = w.shape
            b = self.sd.get(name + ".bias")
            ent = (pack_taps([w.cpu()], K, N).to(self.dev), None if b is None else b.float().contiguous().to(self.dev),
                   N, K)
            self._packed[name] = ent
        return ent

    def __call__(self, x: torch.Tensor, name: str, bias: bool = True,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
        wp, b, N, K = self._pack(name)
        assert x.shape[-1] == K, (name, x.shape, K)
        lead = x.shape[:-1]
        a = x.reshape(-1, K).to(torch.bfloat16)
        if K % 8 or a.stride(0) != K:
            a = a.contiguous()
        M = a.shape[0]
        y = torch.empty(M, N, dtype=torch.float32, device=self.dev) if out is None else out.view(M, N)
        _hip.check(self.lib.itts_igemm_fwd(
            a.data_ptr(), M * K, K, wp.data_ptr(), _hip.ptr(b if bias else None), None, None, None, y.data_ptr(),
            M * N, N, None, 1, M, K, N, 1, _hip.i32_array([0]), 1, 0, 1.0, 0, _hip.F32, _hip.stream_ptr(self.dev)),
            "itts_igemm_fwd")
        return y.view(*lead, N)

    def subsample(self, mel: torch.Tensor, name: str) -> torch.Tensor:
        """``relu(conv2d(mel^T[:, None], stride 2))`` of Conv2dSubsampling2 (gpt/conformer/subsampling.py:
        164-190) as bf16 [B, To, Fo * C] in (f, c) order (``<name>.out.0`` must be applied with its
        columns permuted to match: ``subsample_linear``)."""
        mel = mel.float()
        if mel.stride(2) != 1:
            mel = mel.contiguous()
        B, nb, T = mel.shape
        w = self.sd[name + ".conv.0.weight"]
        C = w.shape[0]
        To, Fo = (T - 3) // 2 + 1, (nb - 3) // 2 + 1
        y = torch.empty(B, To, Fo * C, dtype=torch.bfloat16, device=self.dev)
        _hip.check(self.lib.itts_cond_subsample(
            mel.data_ptr(), mel.stride(0), mel.stride(1), B, nb, T, w.float().contiguous().data_ptr(),
            self.sd[name + ".conv.0.bias"].float().contiguous().data_ptr(), C, y.data_ptr(),
            _hip.stream_ptr(self.dev)), "itts_cond_subsample")
        return y

    def subsample_linear(self, h: torch.Tensor, name: str, C: int) -> torch.Tensor:
        """``<name>.out.0`` (Linear(C * F -> D), inputs in (c, f) order in the reference) on the (f, c)
        rows of ``subsample``: the weight columns permuted once."""
        key = name + ".out.0.fc"
        if key + ".weight" not in self.sd:
            w = self.sd[name + ".out.0.weight"].float()
            D, K = w.shape
            self.register(key, w.view(D, C, K // C).transpose(1, 2).reshape(D, K).contiguous(),
                          self.sd.get(name + ".out.0.bias"))
        return self.splitk(h, key)

    def splitk(self, x: torch.Tensor, name: str) -> torch.Tensor:
        """``bank(x, name)`` for a long reduction over few row tiles (K = 25088 over ~8k rows fills only
        64 workgroups): the K columns in nsplit chunks as a batch of GEMMs (``itts_igemm_splitk``), then
        a fixed-order sum + bias -- enough workgroups for the 256 CUs, rows still independent."""
        w = self.sd[name + ".weight"]
        N, K = w.shape
        lead = x.shape[:-1]
        a = x.reshape(-1, K).to(torch.bfloat16)
        if a.stride(0) != K or a.stride(1) != 1:
            a = a.contiguous()
        M = a.shape[0]
        tiles = -(-M // 256) * -(-N // 256)
        ns = next((n for n in (8, 4, 2) if K % (64 * n) == 0 and K // n >= 1024 and tiles * n <= 1024), 1)
        if ns == 1 or N % 4:
            return self(x, name)
        ent = self._packed.get((name, ns))
        if ent is None:
            from ..vocoder.bigvgan import pack_taps
            kc = K // ns
            wc = w.float().cpu()
            chunks = torch.cat([pack_taps([wc[:, i * kc:(i + 1) * kc].contiguous()], kc, N).reshape(-1)
                                for i in range(ns)]).to(self.dev)
            b = self.sd.get(name + ".bias")
            ent = self._packed[(name, ns)] = (chunks, None if b is None else b.float().contiguous().to(self.dev))
        chunks, b = ent
        part = torch.empty(ns, M, N, dtype=torch.float32, device=self.dev)
        y = torch.empty(M, N, dtype=torch.float32, device=self.dev)
        _hip.check(self.lib.itts_igemm_splitk(a.data_ptr(), K, M, K, chunks.data_ptr(), ns, N, _hip.ptr(b),
                                              part.data_ptr(), y.data_ptr(), _hip.stream_ptr(self.dev)),
                   "itts_igemm_splitk")
        return y.view(*lead, N)

    def glu_dwconv(self, a: torch.Tensor, name: str, eps: float = 1e-5) -> torch.Tensor:
        """ConvolutionModule's GLU -> depthwise_conv -> norm (LayerNorm) -> SiLU
        (gpt/conformer_encoder.py:108-167) of a = pointwise_conv1 output [B, T, 2C] f32 -> bf16 [B, T, C]."""
        if a.stride(-1) != 1 or a.stride(1) != a.shape[-1] or a.stride(0) != a.shape[1] * a.shape[2]:
            a = a.contiguous()
        B, T, C2 = a.shape
        C = C2 // 2
        w = self.sd[name + ".depthwise_conv.weight"]
        K = w.shape[-1]
        key = name + ".depthwise_conv.weight_t"
        if key not in self.sd:  # [K][C]: 16-B weight loads per tap in the LDS-tiled kernel
            self.sd[key] = w.float().reshape(C, K).t().contiguous()
        y = torch.empty(B, T, C, dtype=torch.bfloat16, device=self.dev)
        _hip.check(self.lib.itts_cond_glu_dwconv(
            a.data_ptr(), C2, B, T, C, w.float().reshape(C, K).contiguous().data_ptr(),
            self.sd[name + ".depthwise_conv.bias"].float().contiguous().data_ptr(), K,
            self.sd[name + ".norm.weight"].float().contiguous().data_ptr(),
            self.sd[name + ".norm.bias"].float().contiguous().data_ptr(), eps, y.data_ptr(), C,
            _hip.ptr(self.sd[key] if self.tiled else None), _hip.stream_ptr(self.dev)), "itts_cond_glu_dwconv")
        return y
