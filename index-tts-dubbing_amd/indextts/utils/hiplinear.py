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

    def __call__(self, x: torch.Tensor, name: str, bias: bool = True, out: Optional[torch.Tensor] = None,
                 act: int = 0, bf16_out: bool = False, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """y = act(x @ W^T + b) (+ residual); act 1 = gelu_tanh, 2 = SiLU; bf16_out: bf16 y (the next
        GEMM's operand); residual (f32, contiguous, may be ``out`` itself: y += in place)."""
        wp, b, N, K = self._pack(name)
        assert x.shape[-1] == K, (name, x.shape, K)
        lead = x.shape[:-1]
        a = x.reshape(-1, K).to(torch.bfloat16)
        if K % 8 or a.stride(0) != K:
            a = a.contiguous()
        M = a.shape[0]
        dt = torch.bfloat16 if bf16_out else torch.float32
        y = torch.empty(M, N, dtype=dt, device=self.dev) if out is None else out.view(M, N)
        assert y.dtype == dt and y.is_contiguous()
        r = None
        if residual is not None:
            r = residual.view(M, N)
            assert r.dtype == torch.float32 and r.is_contiguous() and not bf16_out
        _hip.check(self.lib.itts_igemm_fwd(
            a.data_ptr(), M * K, K, wp.data_ptr(), _hip.ptr(b if bias else None), None, _hip.ptr(r), None,
            y.data_ptr(), M * N, N, None, 1, M, K, N, 1, _hip.i32_array([0]), 1, 0, 1.0, act,
            _hip.BF16 if bf16_out else _hip.F32, _hip.stream_ptr(self.dev)), "itts_igemm_fwd")
        return y.view(*lead, N)

    def ln(self, x: torch.Tensor, name: str) -> torch.Tensor:
        """LayerNorm(eps 1e-5) of the rows of x [..., D] f32 -> bf16 (the next GEMM's operand), one
        kernel (itts_layernorm_rows) instead of LayerNorm + cast."""
        D = x.shape[-1]
        xr = x.reshape(-1, D)
        assert xr.stride(1) == 1
        y = torch.empty(xr.shape[0], D, dtype=torch.bfloat16, device=self.dev)
        _hip.check(self.lib.itts_layernorm_rows(xr.data_ptr(), xr.stride(0), None, y.data_ptr(), D, xr.shape[0], D,
                                                self.sd[name + ".weight"].data_ptr(), self.sd[name + ".bias"].data_ptr(),
                                                None, None, _hip.BF16, _hip.stream_ptr(self.dev)), "itts_layernorm_rows")
        return y.view(*x.shape)

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
        # the split count depends on K only (never on M, the rows of every prompt in the batch), so each
        # output's reduction order -- and a prompt's conditioning -- is the same in any batch
        ns = next((n for n in (8, 4, 2) if K % (64 * n) == 0 and K // n >= 1024), 1)
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

    def rel_attn(self, x: torch.Tensor, name: str, heads: int, mask: torch.Tensor, pos_emb: torch.Tensor,
                 residual: Optional[torch.Tensor] = None):
        """RelPositionMultiHeadedAttention (gpt/conformer/attention.py:235-312) of x [B, T, C] f32 with
        key mask [B, 1, T] (a valid prefix per row): q/k/v as one fused GEMM, the attention in
        ``itts_cond_rel_attn`` (row-independent), linear_out on its bf16 output."""
        B, T, C = x.shape
        key = name + ".linear_qkv"
        if key + ".weight" not in self.sd:
            self.register(key, torch.cat([self.sd[f"{name}.linear_{c}.weight"] for c in "qkv"], 0).contiguous(),
                          torch.cat([self.sd[f"{name}.linear_{c}.bias"] for c in "qkv"], 0).contiguous())
        assert C == 64 * heads, "head dim 64"
        qkv = self(x, key)
        pos = torch.nn.functional.linear(pos_emb[0], self.sd[name + ".linear_pos.weight"]).contiguous()
        lens = mask.reshape(B, -1).sum(-1, dtype=torch.int32)
        out = torch.empty(B, T, C, dtype=torch.bfloat16, device=self.dev)
        _hip.check(self.lib.itts_cond_rel_attn(
            qkv.data_ptr(), 3 * C, pos.data_ptr(), C, self.sd[name + ".pos_bias_u"].contiguous().data_ptr(),
            self.sd[name + ".pos_bias_v"].contiguous().data_ptr(), lens.data_ptr(), B, T, heads, 1.0 / 8.0,
            out.data_ptr(), C, _hip.BF16, _hip.stream_ptr(self.dev)), "itts_cond_rel_attn")
        return self(out, name + ".linear_out", out=residual, residual=residual)

    def cross_attn(self, q: torch.Tensor, kv: torch.Tensor, key_mask: torch.Tensor, heads: int, scale: float):
        """PerceiverResampler attention (gpt/perceiver.py:111-150): q [B, 32, H*64] f32, kv [B, nk, 2*H*64]
        (k | v halves, to_kv's chunk order), key_mask [B, nk] bool -> [B, 32, H*64] f32 (itts_cross_attn,
        one workgroup per (head, prompt): a prompt's conds do not depend on the batch)."""
        q, kv = q.float().contiguous(), kv.float().contiguous()
        B, n, inner = q.shape
        nk = kv.shape[1]
        km = key_mask.to(torch.uint8).contiguous()
        out = torch.empty(B, n, inner, dtype=torch.float32, device=self.dev)
        _hip.check(self.lib.itts_cross_attn(
            q.data_ptr(), n * inner, inner, kv.data_ptr(), kv.data_ptr() + 4 * inner, nk * 2 * inner, 2 * inner,
            km.data_ptr(), B, n, nk, heads, float(scale), out.data_ptr(), n * inner, inner,
            _hip.stream_ptr(self.dev)), "itts_cross_attn")
        return out

    # ---------------- ECAPA channel-last (vocoder/ecapa.py speaker_embedding_cl) ----------------
    def pad_rows(self, x: torch.Tensor, pad: int, reflect: bool = True, x2: Optional[torch.Tensor] = None,
                 cp: Optional[int] = None) -> torch.Tensor:
        """bf16 [B, T + 2 pad, cp] of the f32 rows x (+ x2) [B, T, C] (unit channel stride), reflect or
        zero padded in time, channels beyond C zero."""
        B, T, C = x.shape
        cp = cp or (C + 7) // 8 * 8
        assert x.stride(2) == 1 and (x2 is None or (x2.shape == x.shape and x2.stride(2) == 1))
        y = torch.empty(B, T + 2 * pad, cp, dtype=torch.bfloat16, device=self.dev)
        _hip.check(self.lib.itts_pad_rows_bf16(
            x.data_ptr(), x.stride(0), x.stride(1), _hip.ptr(x2), 0 if x2 is None else x2.stride(0),
            0 if x2 is None else x2.stride(1), B, T, C, pad, 1 if reflect else 0, cp, y.data_ptr(),
            _hip.stream_ptr(self.dev)), "itts_pad_rows_bf16")
        return y

    def conv_taps(self, xp: torch.Tensor, name: str, dilation: int, out: Optional[torch.Tensor] = None):
        """conv1d (weight [Cout, Cin, k], bias) over the padded bf16 rows xp [B, Tp, Cp] -> f32
        [B, Tp, Cout]; rows [0, Tp - dilation (k - 1)) are the valid ("same") outputs."""
        B, Tp, Cp = xp.shape
        key = ("taps", name)
        ent = self._packed.get(key)
        if ent is None:
            from ..vocoder.bigvgan import pack_taps
            w = self.sd[name + ".weight"].float().cpu()
            co, ci, k = w.shape
            wp = torch.zeros(co, Cp, k)
            wp[:, :ci] = w
            ent = self._packed[key] = (pack_taps([wp[:, :, j].contiguous() for j in range(k)], Cp, co).to(self.dev),
                                       self.sd[name + ".bias"].float().contiguous().to(self.dev), co, k)
        wpk, b, co, k = ent
        y = torch.empty(B, Tp, co, dtype=torch.float32, device=self.dev) if out is None else out
        _hip.check(self.lib.itts_igemm_fwd(
            xp.data_ptr(), Tp * Cp, Cp, wpk.data_ptr(), b.data_ptr(), None, None, None, y.data_ptr(), y.stride(0),
            y.stride(1), None, B, Tp, Cp, co, k, _hip.i32_array([j * dilation for j in range(k)]), 1, 0, 1.0, 0,
            _hip.F32, _hip.stream_ptr(self.dev)), "itts_igemm_fwd")
        return y

    def relu_bn(self, x: torch.Tensor, name: str, out: Optional[torch.Tensor] = None, eps: float = 1e-5):
        """BatchNorm1d(eval)(relu(x)) over the channels of x [B, T, C] (unit channel stride), as one
        folded affine map; out may be x itself or a strided view."""
        ent = self._packed.get(("bn", name))
        if ent is None:
            sc = self.sd[name + ".weight"].float() / torch.sqrt(self.sd[name + ".running_var"].float() + eps)
            ent = self._packed[("bn", name)] = (sc.contiguous(),
                                               (self.sd[name + ".bias"].float() -
                                                self.sd[name + ".running_mean"].float() * sc).contiguous())
        sc, sh = ent
        B, T, C = x.shape
        y = torch.empty(B, T, C, dtype=torch.float32, device=self.dev) if out is None else out
        _hip.check(self.lib.itts_relu_affine_rows(x.data_ptr(), x.stride(0), x.stride(1), B, T, C, sc.data_ptr(),
                                                  sh.data_ptr(), y.data_ptr(), y.stride(0), y.stride(1),
                                                  _hip.stream_ptr(self.dev)), "itts_relu_affine_rows")
        return y

    def tdnn(self, x: torch.Tensor, name: str, dilation: int = 1, x2: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """TDNNBlock = BN(ReLU(conv(x (+ x2)))) with speechbrain's reflect "same" padding, channel-last."""
        w = self.sd[name + ".conv.conv.weight"]
        k = w.shape[-1]
        T = x.shape[1]
        if k == 1 and x2 is None:
            y = self(x, name + ".conv.conv")
        else:
            y = self.conv_taps(self.pad_rows(x, dilation * (k - 1) // 2, True, x2), name + ".conv.conv", dilation)
            y = y[:, :T]
        return self.relu_bn(y, name + ".norm.norm", out=out)

    def time_stats(self, x: torch.Tensor, logits: Optional[torch.Tensor] = None, want_std: bool = True,
                   eps: float = 1e-12):
        """(mean, std) over time of x [B, T, C] f32 with softmax_t(logits [B, T, C]) or uniform weights;
        one thread per (utterance, channel), row-independent (itts_time_stats)."""
        B, T, C = x.shape
        assert x.stride(2) == 1 and (logits is None or (logits.shape == x.shape and logits.stride(2) == 1))
        mean = torch.empty(B, C, dtype=torch.float32, device=self.dev)
        std = torch.empty(B, C, dtype=torch.float32, device=self.dev) if want_std else None
        _hip.check(self.lib.itts_time_stats(
            x.data_ptr(), x.stride(0), x.stride(1), _hip.ptr(logits), 0 if logits is None else logits.stride(0),
            0 if logits is None else logits.stride(1), B, T, C, eps, mean.data_ptr(), _hip.ptr(std),
            _hip.stream_ptr(self.dev)), "itts_time_stats")
        return mean, std
