"""UnifiedVoice speech-token GPT on the HIP C-ABI: prefill, KV-cached greedy decode, latent pass.

Host mirror of ``UnifiedVoice.inference_speech`` (reference ``indextts/gpt/model.py:655-708``) and
``UnifiedVoice.forward(..., return_latent=True)`` (``:521-589``) for a batch of utterances.

Two numeric modes:
  * ``bf16`` (product): bf16 weights, bf16 GEMM operands with f32 accumulation (MFMA), f32
    residual stream / LayerNorm / softmax / logits, bf16 KV cache.
  * ``f32`` (verification): f32 weights/activations/cache through exact-f32 VALU GEMMs; used to
    show bit-exact greedy ids against the fp32 reference.

HBM layout (per engine, batch capacity B): residual x [B, D] f32; GEMM operands padded to 32-row
MFMA tiles; KV cache [layers][B][heads][Smax][64]; decode state (token counter, seen-id bitmap,
done flags, codes) lives on the device so one captured hipGraph replays every step.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import os
import warnings
from typing import List, Optional

import numpy as np
import torch

from .. import _hip
from .conditioning import get_conditioning


def _t(v):
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))


def _host(v, dtype=torch.float32):
    """contiguous CPU copy (the packers are host functions of the C ABI)"""
    return _t(v).detach().to("cpu", dtype).contiguous()


def _ptr_or_none(t):
    return None if t is None else t.data_ptr()


def pack_frag(w_t, cols: int) -> torch.Tensor:
    """W^T [N, K] (f32, rounded to bf16 here, or bf16) -> MFMA fragment order on the host through
    itts_gpt_pack_frag (include/itts_hip.h): cols 32 -> [N/32][K/16][64 lanes][8] (lane 32h + r holds
    W^T[32nt + r][16s + 8h : +8]), cols 16 -> [N/16][K/32][64][8] (lane 16q + c holds W^T[16nt + c][32s + 8q
    : +8]); N zero-padded to a multiple of cols."""
    lib = _hip.load()
    w = _t(w_t).detach().cpu()
    w = w.contiguous() if w.dtype == torch.bfloat16 else w.float().contiguous()
    N, K = w.shape
    ks = 16 if cols == 32 else 32
    assert K % ks == 0
    Np = (N + cols - 1) // cols * cols
    out = torch.empty(Np * K, dtype=torch.bfloat16)
    _hip.check(lib.itts_gpt_pack_frag(w.data_ptr(), _hip.BF16 if w.dtype == torch.bfloat16 else _hip.F32, N, K, cols,
                                      out.data_ptr()), "itts_gpt_pack_frag")
    return out.view(Np // cols, K // ks, 64 // cols, cols, 8)


def pack_skinny(w_t: torch.Tensor) -> torch.Tensor:
    """32-column fragment order (itts_decode_gemm; attn.c_proj / mlp.c_proj split-K, mel_head)."""
    return pack_frag(w_t, 32)


def pack_skinny16(w_t: torch.Tensor) -> torch.Tensor:
    """16-column fragment order (itts_decode_gemm16 / 16x)."""
    return pack_frag(w_t, 16)


def fold_ln_weights(w_io, bias, ln, device, keep_wt: bool = False):
    """Operands of itts_decode_gemm16x for HF Conv1D weight ``w_io`` [in=K, out=N] (+ bias [N]) fed by
    LayerNorm ``ln`` = (g, b) (None: no LayerNorm), through itts_gpt_fold_ln: W' = diag(g) W rounded to
    bf16 and packed on 16-column tiles, u = column sums of the ROUNDED W' (so the kernel's mean term
    cancels exactly what its MFMAs accumulated), c = b^T W + bias (float64 accumulation).
    keep_wt: also return the host bf16 W'^T [N, K] (pack_qkv12's input)."""
    lib = _hip.load()
    w, bs = _host(w_io), _host(bias)
    K, N = w.shape
    g, b = (None, None) if ln is None else (_host(ln[0]), _host(ln[1]))
    wt = torch.empty(N, K, dtype=torch.bfloat16)
    u = None if ln is None else torch.empty(N)
    c = torch.empty(N)
    _hip.check(lib.itts_gpt_fold_ln(w.data_ptr(), bs.data_ptr(), _ptr_or_none(g), _ptr_or_none(b), K, N, wt.data_ptr(),
                                    _ptr_or_none(u), c.data_ptr()), "itts_gpt_fold_ln")
    out = {"w16": pack_skinny16(wt).to(device), "u": None if u is None else u.to(device), "c": c.to(device),
           "N": N, "K": K}
    if keep_wt:
        out["wt"], out["u_host"], out["c_host"] = wt, u, c
    return out


def pack_qkv12(wx_qkv, n_head: int = 16):
    """Persistent-layer c_attn operands (gpt_layer.hip) through itts_gpt_pack_qkv12: workgroup b = 8j + c
    computes 12 columns of head h = 2c + j/16 -- columns 12*(j%16) .. +11 of that head's [q | k | v] 192 --
    from the SAME rounded W' = diag(ln_1.g) W and fold terms u / c as itts_decode_gemm16x (``wx_qkv`` from
    fold_ln_weights(..., keep_wt=True)), in 16x16x32 B-fragment order without the 4 unused columns:
    W12 [256][32 k-steps][4][12][8] bf16, uc [256][2][12] f32."""
    lib = _hip.load()
    wt = wx_qkv["wt"]
    N, K = wt.shape
    w12 = torch.empty(256, K // 32, 4, 12, 8, dtype=torch.bfloat16)
    uc = torch.empty(256, 2, 12)
    _hip.check(lib.itts_gpt_pack_qkv12(wt.data_ptr(), wx_qkv["u_host"].data_ptr(), wx_qkv["c_host"].data_ptr(), K,
                                       n_head, w12.data_ptr(), uc.data_ptr()), "itts_gpt_pack_qkv12")
    dev = wx_qkv["u"].device
    return {"w12": w12.to(dev), "uc": uc.to(dev)}


# the persistent decode layers are the default (C3 decode step 710 vs 765 us on the launch chain,
# profiles/pl_trace_r04c.txt); ITTS_PL=0 selects the chain.  Their per-step counter / granule reset is a
# kernel: as a hipMemsetAsync node it let 30 of 64 reused-lane cues decode wrong data
# (profiles/lf_stress_memset.txt vs lf_stress_default.txt)
PL_DEFAULT = "1"


class _Layer:
    pass


class HipGPT:
    def __init__(self, state_dict, cfg_gpt, device="cuda", dtype: str = "bf16", max_batch: int = 32,
                 max_kv: Optional[int] = None):
        assert dtype in ("bf16", "f32")
        self.lib = _hip.load()
        self.cfg = g = cfg_gpt
        self.dev = torch.device(device)
        self.mode = dtype
        self.D, self.L, self.H = int(g.model_dim), int(g.layers), int(g.heads)
        assert self.D == 64 * self.H, "kernels assume head size 64"
        self.V = int(g.number_mel_codes)
        self.Vp = (self.V + 15) // 16 * 16  # logits / seen-flag row pitch (vectorised sampler loads)
        self.start_text, self.stop_text = int(g.start_text_token), int(g.stop_text_token)
        self.start_mel, self.stop_mel = int(g.start_mel_token), int(g.stop_mel_token)
        self.max_kv = int(max_kv or (32 + int(g.max_text_tokens) + 2 + 1 + int(g.max_mel_tokens)))
        sd = {k: _t(v) for k, v in state_dict.items()}
        dev = self.dev
        f32 = lambda k: sd[k].float().to(dev).contiguous()  # noqa: E731
        self.sd_cond = {k: v.float().to(dev) for k, v in sd.items()
                        if k.startswith(("conditioning_encoder", "perceiver_encoder"))}
        self.text_emb, self.text_pos = f32("text_embedding.weight"), f32("text_pos_embedding.emb.weight")
        self.mel_emb, self.mel_pos = f32("mel_embedding.weight"), f32("mel_pos_embedding.emb.weight")
        self.ln_f = (f32("gpt.ln_f.weight"), f32("gpt.ln_f.bias"))
        self.final_norm = (f32("final_norm.weight"), f32("final_norm.bias"))
        # decode-step variants (bf16 product mode), measured at B=32 (scratch/ubench_fusions.py):
        #  * c_fc on 16-column tiles (itts_decode_gemm16): 6.2 -> 5.5 us, on by default (ITTS_DG16=0: off);
        #    mel_head stays on 32-column tiles (16-column: 9.5 -> 14.8 us, 513 workgroups too many)
        #  * attn.c_proj fused into the attention kernel (itts_attn_decode_proj, one f32 partial per
        #    head): 22.7 us vs 17.0 us for attention + the split-K GEMM at S=283 -- W's 128 KiB per
        #    workgroup need 256 VGPRs (1 workgroup per CU; at 2 it spills), so off by default
        #    (ITTS_ATTN_PROJ=1: on)
        self.fuse_o = dtype == "bf16" and self.D <= 1024 and os.environ.get("ITTS_ATTN_PROJ", "0") == "1"
        self.use_dg16 = dtype == "bf16" and os.environ.get("ITTS_DG16", "1") != "0"
        #  * LayerNorm folded into the consumer GEMMs + residual epilogues (itts_decode_gemm16x): five
        #    launches per layer instead of seven (ITTS_LN_FOLD=0: the split-K + reduce/LN path)
        self.fold = dtype == "bf16" and not self.fuse_o and os.environ.get("ITTS_LN_FOLD", "1") != "0"
        #  * mlp.c_proj: split-K 8 + reduce launch (default) or one full-K launch of 64 workgroups with
        #    the residual epilogue (ITTS_PROJ_FULLK=1)
        self.proj_fullk = self.fold and os.environ.get("ITTS_PROJ_FULLK", "0") == "1"
        #  * the whole step as ONE C-ABI call, itts_gpt_decode_step (gpt_step.hip), launching the same
        #    kernels as _decode_step_fold (ITTS_CSTEP=0: the Python launch sequence, kept as the test
        #    reference); multi-role launches and a side-stream K/V prefetch were measured slower
        #    (profiles/ubench_fused_r02.txt)
        self.cstep = self.fold and os.environ.get("ITTS_CSTEP", "1") != "0"
        #  * every layer of the step as ONE persistent launch (itts_gpt_decode_steps_pl, gpt_layer.hip) for
        #    1..128 rows of the IndexTTS-1.5 shape (beam lineage included) on a 256-CU device; bit-identical
        #    to the launch chain (ITTS_PL=0: the chain)
        self.pl = self.cstep and os.environ.get("ITTS_PL", PL_DEFAULT) != "0" and self.D == 1024 and self.H == 16
        self.layers: List[_Layer] = []
        for i in range(self.L):
            p = f"gpt.h.{i}"
            ly = _Layer()
            ly.ln1, ly.ln2 = (f32(p + ".ln_1.weight"), f32(p + ".ln_1.bias")), (f32(p + ".ln_2.weight"), f32(p + ".ln_2.bias"))
            ly.b = {n: f32(f"{p}.{k}.bias") for n, k in
                    (("qkv", "attn.c_attn"), ("o", "attn.c_proj"), ("fc", "mlp.c_fc"), ("proj", "mlp.c_proj"))}
            ly.w = {}
            for n, k in (("qkv", "attn.c_attn"), ("o", "attn.c_proj"), ("fc", "mlp.c_fc"), ("proj", "mlp.c_proj")):
                wt = sd[f"{p}.{k}.weight"].float().t().contiguous()  # HF Conv1D [in, out] -> [out, in]
                ly.w[n] = self._pack(wt, sk16=n == "fc")
            if self.fold:  # itts_decode_gemm16x operands (LayerNorm folded / residual epilogue)
                ly.wx = {}
                for n, k, ln in (("qkv", "attn.c_attn", ly.ln1), ("o", "attn.c_proj", None),
                                 ("fc", "mlp.c_fc", ly.ln2), ("proj", "mlp.c_proj", None)):
                    ly.wx[n] = fold_ln_weights(sd[f"{p}.{k}.weight"], sd[f"{p}.{k}.bias"],
                                               None if ln is None else (sd[f"{p}.ln_{1 if n == 'qkv' else 2}.weight"],
                                                                        sd[f"{p}.ln_{1 if n == 'qkv' else 2}.bias"]),
                                               dev, keep_wt=n == "qkv")
                if self.pl:
                    ly.pl = pack_qkv12(ly.wx["qkv"], self.H)
                for key in ("wt", "u_host", "c_host"):
                    ly.wx["qkv"].pop(key, None)
            if self.fuse_o:  # attn.c_proj in HF Conv1D [in, out] order (bf16) for the fused attention
                ly.wo_io = sd[f"{p}.attn.c_proj.weight"].float().to(torch.bfloat16).contiguous().to(dev)
            self.layers.append(ly)
        self.head_w = self._pack(sd["mel_head.weight"].float().contiguous(), igemm=False)
        self.head_b = f32("mel_head.bias")
        if self.fold:
            self._cweights = self._c_weights()
        if self.pl:
            self._plw = (_hip.GptPlLayerW * self.L)(*[_hip.GptPlLayerW(ly.pl["w12"].data_ptr(), ly.pl["uc"].data_ptr())
                                                     for ly in self.layers])
            n = int(self.lib.itts_gpt_pl_scratch_bytes())
            # zero-filled = armed (epoch 0); never reset between steps or calls, only after a hand-off
            # timeout (_pl_recover).  torch's allocations are 256-B aligned.
            self._pl_scratch = torch.zeros(n // 4 + 64, dtype=torch.float32, device=dev)
        self._pl_block = 0     # > 0: decode on the launch chain (launch_chain(); another grid may share the CUs)
        self._pl_strikes = 0   # hand-off timeouts so far; PL_MAX_STRIKES of them turn the persistent path off
        self._pl_ran = False   # the last generate ran persistent layers (their error word is checked after it)
        self._lanes = {}  # lane index -> decode state, captured graph, stream
        self.step_events = None  # set to a list to time every decode step with HIP events (bench.py)
        # beams + step_events: the kv_rows lineage table is snapshotted after every replay, and each step's
        # key count becomes the DISTINCT (cache row, position) pairs its beams read (bench.py roofline)
        self.beam_lineage = None
        self.logits_trace = None  # set to a list to record every step's raw logits [B, V] (tests)
        # set to a list to record every beam step's state after its selection (tests): one step per replay, then
        # (codes [R, steps], beam scores [R], utterances done [B]) on the host
        self.beam_trace = None
        # algorithmic HBM bytes of one decode step: every weight byte once (+ per-key KV bytes)
        eb = 2 if dtype == "bf16" else 4
        self.step_weight_bytes = sum(eb * ly.w[n]["N"] * ly.w[n]["K"] for ly in self.layers for n in ly.w) \
            + eb * self.head_w["N"] * self.head_w["K"]
        self.kv_bytes_per_key = self.L * self.H * 64 * 2 * eb  # the K and V rows of one key, all layers

    # ---------------- weights ----------------
    def _pack(self, wt: torch.Tensor, igemm: bool = True, sk16: bool = False):
        """wt: [N, K] f32 -> dict of device copies for the kernels of this mode."""
        N, K = wt.shape
        if self.mode == "f32":
            return {"f32": wt.to(self.dev), "N": N, "K": K}
        out = {"sk": pack_skinny(wt).to(self.dev), "N": N, "K": K}
        if sk16 and self.use_dg16 and K % 32 == 0:
            out["sk16"] = pack_skinny16(wt).to(self.dev)
        if igemm:
            from ..vocoder.bigvgan import pack_taps
            out["ig"] = pack_taps([wt], K, N).to(self.dev)
        return out

    # ---------------- conditioning + inputs ----------------
    @torch.no_grad()
    def conditioning(self, mel: torch.Tensor, mel_lengths=None, fast: bool = False) -> torch.Tensor:
        """conds [B, 32, D] of prompt mels [B, 100, T].  fast=True: the linear layers on the bf16 MFMA
        implicit GEMM (utils/hiplinear.py; the reference's fp16 mode runs this under autocast,
        infer.py:572-586); fast=False: f32 torch (the exact-f32 verification mode and the oracle tests).
        Convolutions are GEMMs (utils/convgemm.py): run-to-run identical without MIOpen."""
        lin = None
        if fast:
            if getattr(self, "_cond_bank", None) is None:
                from ..utils.hiplinear import HipLinearBank
                self._cond_bank = HipLinearBank(self.sd_cond, self.dev)
            lin = self._cond_bank
        return get_conditioning(self.sd_cond, self.cfg, mel.to(self.dev).float(),
                                None if mel_lengths is None else mel_lengths.to(self.dev), lin=lin)

    def prepare_inputs(self, conds: torch.Tensor, text_ids: torch.Tensor):
        """``prepare_gpt_inputs`` (gpt/model.py:591-654): strip ids 0/1, [0]+ids+[1], left zero pad.
        -> emb [B, s+1, D] f32 (incl. the start-mel position), pad [B] int32, s."""
        B, L = text_ids.shape
        conds = conds.to(self.dev).float()
        ncond = conds.shape[1]
        s = ncond + L + 2
        D, dev = self.D, self.dev
        # vectorised over rows (no host sync): kept ids packed to the right end of the [B, L+2] text
        # block behind the start id, the stop id last; rows left-padded with zero embeddings
        ids = text_ids.to(dev).long()
        keep = (ids != self.stop_text) & (ids != self.start_text)
        cnt = keep.sum(1)                                           # [B]
        pad = L - cnt                                               # = L + 2 - (cnt + 2)
        rank = torch.cumsum(keep.long(), 1) - 1                     # position among the kept ids
        dst = pad[:, None] + 1 + rank                               # column in the [L+2] text block
        tok = torch.full((B, L + 2), self.start_text, dtype=torch.long, device=dev)
        tok.scatter_(1, torch.where(keep, dst, torch.full_like(dst, L + 1)), torch.where(keep, ids, torch.full_like(ids, self.stop_text)))
        tok[torch.arange(B, device=dev), pad + cnt + 1] = self.stop_text
        col = torch.arange(L + 2, device=dev)[None, :]
        tpos = (col - pad[:, None]).clamp(min=0)                    # text positions restart at 0 per row
        te = self.text_emb[tok] + self.text_pos[tpos]               # [B, L+2, D]
        cb = conds.expand(B, -1, -1) if conds.shape[0] == 1 else conds
        # the conditioning block sits right before the row's text: rows [pad, pad + ncond)
        blk = torch.cat([cb, te], 1)                                # [B, ncond + L + 2, D] (unpadded order)
        j = torch.arange(s, device=dev)[None, :]                    # output column
        srcc = j - pad[:, None]                                     # source column (negative: padding)
        valid = srcc >= 0
        # the text block's padded prefix columns of `te` must be skipped: source index in blk
        srcb = torch.where(srcc < ncond, srcc, ncond + pad[:, None] + (srcc - ncond))
        g = torch.gather(blk, 1, srcb.clamp(min=0, max=ncond + L + 1)[..., None].expand(B, s, D))
        emb = torch.zeros(B, s + 1, D, device=dev)
        emb[:, :s] = g * valid[..., None]
        emb[:, s] = self.mel_emb[self.start_mel] + self.mel_pos[0]
        return emb, pad.int(), s

    # ---------------- GEMM dispatch ----------------
    def _gemm(self, A, w, Y, bias=None, gelu=False, residual=False):
        """Full-sequence GEMM Y = A @ W^T (+bias)(gelu)(+Y if residual), A [M, K]: the MFMA implicit
        GEMM in bf16 mode, the exact-f32 GEMM in f32 mode (which also serves its decode step)."""
        M, K = A.shape
        N = w["N"]
        st = _hip.stream_ptr()
        if self.mode == "f32":
            _hip.check(self.lib.itts_gemm_f32(A.data_ptr(), A.stride(0), w["f32"].data_ptr(), K, M, N, K,
                                              _hip.ptr(bias), int(gelu), Y.data_ptr() if residual else None,
                                              Y.data_ptr(), Y.stride(0), st), "itts_gemm_f32")
            return
        _hip.check(self.lib.itts_igemm_fwd(A.data_ptr(), M * K, K, w["ig"].data_ptr(), _hip.ptr(bias), None,
                                           Y.data_ptr() if residual else None, None, Y.data_ptr(), M * N,
                                           Y.stride(0), None, 1, M, K, N, 1, _hip.i32_array([0]), 1, 0, 1.0,
                                           int(gelu), _hip.dtype_code(Y), st), "itts_igemm_fwd")

    def _ln(self, x, y, ln, ln2=None, idx=None, M=None):
        M = x.shape[0] if M is None else M
        _hip.check(self.lib.itts_layernorm_rows(
            x.data_ptr(), x.stride(0), _hip.ptr(idx), y.data_ptr(), y.stride(0), M, self.D, ln[0].data_ptr(),
            ln[1].data_ptr(), None if ln2 is None else ln2[0].data_ptr(), None if ln2 is None else ln2[1].data_ptr(),
            _hip.dtype_code(y), _hip.stream_ptr()), "itts_layernorm_rows")

    @property
    def act_dtype(self):
        return torch.bfloat16 if self.mode == "bf16" else torch.float32

    # ---------------- full-sequence forward (prefill + latent pass) ----------------
    # the sequence passes as ONE C-ABI call each (itts_gpt_forward_rows / itts_gpt_prefill, gpt_seq.hip:
    # the launch sequence of _forward_rows_py in C++, so a non-Python host can run prefill, decode and
    # the latent pass through the ABI alone); ITTS_CSEQ=0: the Python launch sequence (test reference)
    cseq = os.environ.get("ITTS_CSEQ", "1") != "0"

    def _c_seq_weights(self):
        """ItTsGptSeqWeights (include/itts_hip.h) over this engine's sequence-GEMM weights."""
        if getattr(self, "_cseqw", None) is None:
            L = len(self.layers)
            arr = (_hip.GptSeqLayerW * L)()
            key = "f32" if self.mode == "f32" else "ig"
            for i, ly in enumerate(self.layers):
                arr[i] = _hip.GptSeqLayerW(*[ly.w[n][key].data_ptr() for n in ("qkv", "o", "fc", "proj")],
                                           *[ly.b[n].data_ptr() for n in ("qkv", "o", "fc", "proj")],
                                           ly.ln1[0].data_ptr(), ly.ln1[1].data_ptr(), ly.ln2[0].data_ptr(),
                                           ly.ln2[1].data_ptr())
            w = _hip.GptSeqWeights(L, self.D, self.H, _hip.F32 if self.mode == "f32" else _hip.BF16, arr,
                                   self.ln_f[0].data_ptr(), self.ln_f[1].data_ptr(), self.final_norm[0].data_ptr(),
                                   self.final_norm[1].data_ptr(),
                                   self.head_w["f32"].data_ptr() if self.mode == "f32" else None)
            w._layers = arr
            self._cseqw = w
        return self._cseqw

    def _c_head_weights(self):
        """ItTsGptWeights for the prefill's head + sampler (the decode structs in fold mode; f32 mode has
        no packed decode layers, so a struct without them)."""
        if self.fold:
            return self._cweights
        if getattr(self, "_cheadw", None) is None:
            self._cheadw = _hip.GptWeights(self.L, self.D, self.H, self.V, self.Vp, self.start_mel, self.stop_mel, None,
                                           self.ln_f[0].data_ptr(), self.ln_f[1].data_ptr(),
                                           self.final_norm[0].data_ptr(), self.final_norm[1].data_ptr(),
                                           self.head_w["sk"].data_ptr() if "sk" in self.head_w else None,
                                           self.head_b.data_ptr(), self.mel_emb.data_ptr(), self.mel_pos.data_ptr())
        return self._cheadw

    def _seq_workspace(self, M):
        n = int(self.lib.itts_gpt_forward_rows_workspace_bytes(ctypes.byref(self._c_seq_weights()), int(M)))
        return torch.empty(max(n, 1), dtype=torch.uint8, device=self.dev)

    def _forward_rows(self, x, seq_start, seq_len, seq_pad, max_len, cache=None, out_idx=None, out=None):
        """x [M, D] f32 (in place) through all layers (+ out[i] = final_norm(ln_f(x[out_idx[i]])))."""
        if not self.cseq:
            self._forward_rows_py(x, seq_start, seq_len, seq_pad, max_len, cache)
            if out is not None:
                self._ln(x, out.view(-1, self.D), self.ln_f, self.final_norm, idx=out_idx, M=out_idx.numel())
            return x
        M, D = x.shape
        ck = cv = None
        cbs = chs = cls = 0
        cdt = _hip.dtype_code(x) if self.mode == "f32" else _hip.BF16
        if cache is not None:
            ck, cv = cache
            cbs, chs, cls, cdt = ck.stride(1), ck.stride(2), ck.stride(0), _hip.dtype_code(ck)
        ws = self._seq_workspace(M)
        _hip.check(self.lib.itts_gpt_forward_rows(
            ctypes.byref(self._c_seq_weights()), x.data_ptr(), M, seq_start.data_ptr(), seq_len.data_ptr(),
            _hip.ptr(seq_pad), seq_start.numel(), int(max_len), _hip.ptr(ck), _hip.ptr(cv), cbs, chs, cls, cdt,
            _hip.ptr(out_idx), 0 if out is None else int(out_idx.numel()), _hip.ptr(out),
            _hip.dtype_code(out) if out is not None else 0, ws.data_ptr(), _hip.stream_ptr()), "itts_gpt_forward_rows")
        return x

    def _forward_rows_py(self, x, seq_start, seq_len, seq_pad, max_len, cache=None):
        """x [M, D] f32 (modified in place) through all layers; returns x (pre ln_f)."""
        M, D = x.shape
        ad = self.act_dtype
        h = torch.empty(M, D, dtype=ad, device=self.dev)
        qkv = torch.empty(M, 3 * D, dtype=torch.float32, device=self.dev)
        o = torch.empty(M, D, dtype=ad, device=self.dev)
        f = torch.empty(M, 4 * D, dtype=ad, device=self.dev)
        st = _hip.stream_ptr()
        cdt = _hip.dtype_code(cache[0]) if cache is not None else _hip.dtype_code(h)
        for li, ly in enumerate(self.layers):
            self._ln(x, h, ly.ln1)
            self._gemm(h, ly.w["qkv"], qkv, bias=ly.b["qkv"])
            ck = cv = None
            cbs = chs = 0
            if cache is not None:
                ck, cv = cache[0][li], cache[1][li]
                cbs, chs = ck.stride(0), ck.stride(1)
            _hip.check(self.lib.itts_attn_prefill(
                qkv.data_ptr(), 3 * D, seq_start.data_ptr(), seq_len.data_ptr(), _hip.ptr(seq_pad), seq_start.numel(),
                max_len, _hip.ptr(ck), _hip.ptr(cv), cbs, chs, o.data_ptr(), D, self.H, cdt, _hip.dtype_code(o), st),
                "itts_attn_prefill")
            self._gemm(o, ly.w["o"], x, bias=ly.b["o"], residual=True)
            self._ln(x, h, ly.ln2)
            self._gemm(h, ly.w["fc"], f, bias=ly.b["fc"], gelu=True)
            self._gemm(f, ly.w["proj"], x, bias=ly.b["proj"], residual=True)
        return x

    # ---------------- decode state ----------------
    def _alloc_state(self, B: int, max_new: int):
        D, dev = self.D, self.dev
        Mp = (B + 31) // 32 * 32
        ad = self.act_dtype
        cdt = torch.bfloat16 if self.mode == "bf16" else torch.float32
        st = {
            "B": B, "Mp": Mp, "max_new": max_new,
            "x": torch.zeros(B, D, device=dev),
            "h": torch.zeros(Mp, D, dtype=ad, device=dev),
            "qkv": torch.zeros(self.KSPLIT["qkv"] * B * 3 * D, device=dev),  # c_attn split-K slabs [split][B][3D]
            "o": torch.zeros(Mp, D, dtype=ad, device=dev),
            "f": torch.zeros(Mp, 4 * D, dtype=ad, device=dev),
            "ws": torch.zeros(max(8, self.KSPLIT["o"], self.KSPLIT["proj"], self.H) * B * D, device=dev),  # split-K partials [split][B][D]
            "logits": torch.zeros(B, self.Vp, device=dev),  # row pitch Vp (16-B aligned rows)
            "kc": torch.empty(self.L, B, self.H, self.max_kv, 64, dtype=cdt, device=dev),
            "vc": torch.empty(self.L, B, self.H, self.max_kv, 64, dtype=cdt, device=dev),
            "seen": torch.zeros(B, self.Vp, dtype=torch.uint8, device=dev),  # same row pitch as logits
            "done": torch.zeros(B, dtype=torch.uint8, device=dev),
            "codes": torch.full((B, max_new), self.stop_mel, dtype=torch.int32, device=dev),
            "t": torch.zeros(4, dtype=torch.int32, device=dev),
            "pad": torch.zeros(B, dtype=torch.int32, device=dev),  # graph-captured pointer: update in place
        }
        return st

    def _embed_ln(self):
        """LayerNorm the sampler applies to the next token's embedding (h = ln_1(x) of layer 0), or
        none when ln_1 is folded into c_attn (h = bf16 x)."""
        if self.fold:
            return None, None
        return self.layers[0].ln1[0].data_ptr(), self.layers[0].ln1[1].data_ptr()

    def _sample(self, st, col_delta, min_new, penalty):
        smp = st.get("sampling")
        if smp is not None:  # (temperature, top_k, top_p); the seed is device state (t[2:4])
            _hip.check(self.lib.itts_sample_topk_embed(
                st["logits"].data_ptr(), self.Vp, self.V, st["seen"].data_ptr(), st["done"].data_ptr(),
                st["codes"].data_ptr(), st["max_new"], st["t"].data_ptr(), col_delta, int(min_new), self.stop_mel,
                float(penalty), float(smp[0]), int(smp[1]), float(smp[2]), self.mel_emb.data_ptr(),
                self.mel_pos.data_ptr(), 2, self.D, *self._embed_ln(),
                st["x"].data_ptr(), st["h"].data_ptr(), _hip.dtype_code(st["h"]), st["B"],
                _hip.ptr(st.get("forced")), _hip.stream_ptr()), "itts_sample_topk_embed")
            return
        _hip.check(self.lib.itts_sample_embed(
            st["logits"].data_ptr(), self.Vp, self.V, st["seen"].data_ptr(), st["done"].data_ptr(),
            st["codes"].data_ptr(), st["max_new"], st["t"].data_ptr(), col_delta, int(min_new), self.stop_mel,
            float(penalty), self.mel_emb.data_ptr(), self.mel_pos.data_ptr(), 2, self.D,
            *self._embed_ln(), st["x"].data_ptr(),
            st["h"].data_ptr(), _hip.dtype_code(st["h"]), st["B"], _hip.ptr(st.get("forced")), _hip.stream_ptr()),
            "itts_sample_embed")

    def _dgx(self, A, wx, M, Y, epi=0, gelu=False, xh=None, nwaves=8):
        """itts_decode_gemm16x: LayerNorm-folded store epilogue (wx["u"] set) or residual epilogue."""
        _hip.check(self.lib.itts_decode_gemm16x(
            A.data_ptr(), A.stride(0), wx["w16"].data_ptr(), wx["K"], wx["N"], M, _hip.ptr(wx["c"]),
            _hip.ptr(wx["u"]), 1e-5, int(gelu), epi, Y.data_ptr(), Y.stride(0), _hip.dtype_code(Y), _hip.ptr(xh),
            0 if xh is None else xh.stride(0), nwaves, _hip.stream_ptr()), "itts_decode_gemm16x")

    def _c_weights(self):
        """ItTsGptWeights (include/itts_hip.h) over this engine's packed tensors (kept alive by self)."""
        L = len(self.layers)
        arr = (_hip.GptLayerW * L)()
        for i, ly in enumerate(self.layers):
            wx = ly.wx
            arr[i] = _hip.GptLayerW(wx["qkv"]["w16"].data_ptr(), wx["qkv"]["u"].data_ptr(), wx["qkv"]["c"].data_ptr(),
                                    wx["o"]["w16"].data_ptr(), wx["o"]["c"].data_ptr(), wx["fc"]["w16"].data_ptr(),
                                    wx["fc"]["u"].data_ptr(), wx["fc"]["c"].data_ptr(), ly.w["proj"]["sk"].data_ptr(),
                                    ly.b["proj"].data_ptr(), ly.w["o"]["sk"].data_ptr())
        w = _hip.GptWeights(L, self.D, self.H, self.V, self.Vp, self.start_mel, self.stop_mel, arr,
                            self.ln_f[0].data_ptr(), self.ln_f[1].data_ptr(), self.final_norm[0].data_ptr(),
                            self.final_norm[1].data_ptr(), self.head_w["sk"].data_ptr(), self.head_b.data_ptr(),
                            self.mel_emb.data_ptr(), self.mel_pos.data_ptr())
        w._layers = arr  # keep the array alive with the struct
        return w

    def _c_state(self, st):
        """ItTsGptDecodeState over one decode state's tensors (rebuilt per call: `forced` may change)."""
        kv_rows = st.get("kv_rows")
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        return _hip.GptDecodeState(
            st["B"], self.max_kv, st["s"] + 1, st["max_new"], p(st["x"]), p(st["h"]), p(st["qkv"]), p(st["o"]),
            p(st["f"]), p(st["ws"]), p(st["logits"]), p(st["kc"]), p(st["vc"]), p(st["pad"]), p(st["t"]), p(kv_rows),
            0 if kv_rows is None else kv_rows.stride(0), p(st["seen"]), p(st["done"]), p(st["codes"]),
            p(st.get("forced")), int(st["beam"]["K"]) if kv_rows is not None and "beam" in st else 0)

    def _decode_step_c(self, st, min_new, penalty, nsteps=1):
        """bf16 product decode step as ONE C-ABI call (itts_gpt_decode_step, gpt_step.hip): the launches
        of _decode_step_fold, mel_head, token selection, step advance.  Bit-identical to
        _decode_step_fold (tests/test_gpu_cstep.py).  nsteps > 1 (not beams): that many steps in one
        call with one step-counter advance (itts_gpt_decode_steps)."""
        beams = "kv_rows" in st
        smp = st.get("sampling")
        if beams:
            mode = _hip.Sampling(2, 0, 1.0, 1.0, 0, 1.0)
        elif smp is None:
            mode = _hip.Sampling(0, int(min_new), float(penalty), 1.0, 0, 1.0)
        else:
            mode = _hip.Sampling(1, int(min_new), float(penalty), float(smp[0]), int(smp[1]), float(smp[2]))
        cst = self._c_state(st)
        stream = _hip.stream_ptr()
        if self._pl_ok(st):  # every layer one persistent launch (bit-identical to the chain)
            _hip.check(self.lib.itts_gpt_decode_steps_pl(ctypes.byref(self._cweights), self._plw,
                                                         self._pl_scratch.data_ptr(), ctypes.byref(cst),
                                                         ctypes.byref(mode), 1 if beams else int(nsteps), stream),
                       "itts_gpt_decode_steps_pl")
            if beams:
                self._beam_step(st, 1)
                _hip.check(self.lib.itts_step_advance(st["t"].data_ptr(), 1, stream), "itts_step_advance")
            return
        if nsteps > 1:
            assert not beams
            _hip.check(self.lib.itts_gpt_decode_steps(ctypes.byref(self._cweights), ctypes.byref(cst),
                                                      ctypes.byref(mode), int(nsteps), stream), "itts_gpt_decode_steps")
            return
        _hip.check(self.lib.itts_gpt_decode_step(ctypes.byref(self._cweights), ctypes.byref(cst), ctypes.byref(mode),
                                                 stream), "itts_gpt_decode_step")
        if beams:
            self._beam_step(st, 1)
            _hip.check(self.lib.itts_step_advance(st["t"].data_ptr(), 1, stream), "itts_step_advance")

    # rows up to which a step runs on the persistent layers: every shape the kernel supports (<= 128 rows, four
    # row tiles).  Round 5 (row tiles straight-line with exact vmcnt counts, o prefetched) made the multi-tile
    # steps faster than the chain too: greedy 32 / 64 / 96 / 128 rows 664 / 1016 / 1330 / 1649 us per step vs
    # 780 / 1127 / 1452 / 1688 on the chain (profiles/ubench_pl_rows.py, pl_rows_r05rows.txt), and the C5
    # long-form 128-row chunks 1794 / 1829 vs 1784 / 1777 audio-s/s run back to back on them (r05c5_ab.txt;
    # round 4 kept them on the chain, 32 rows was the break-even then).  Beam states (lineage table) up to
    # PL_MAX_BEAM_ROWS: beam3's 96-row step 1330 us vs 1360 on the chain (profiles/r05_b3pl.sh r05u)
    PL_MAX_ROWS = int(os.environ.get("ITTS_PL_MAX_ROWS", "128"))
    PL_MAX_BEAM_ROWS = int(os.environ.get("ITTS_PL_MAX_BEAM_ROWS", "96"))
    BEAM_MAX_KV = 3584  # kKviMax of gpt_attn.hip / gpt_layer.hip (lineage indices staged in LDS)

    @property
    def pl_active(self):
        """persistent layers enabled and not held off by launch_chain()"""
        return self.pl and self._pl_block == 0

    @contextlib.contextmanager
    def launch_chain(self):
        """Decode on the launch chain inside this block.  The persistent grid needs all 256 CUs at once
        (one workgroup per CU): callers that run other kernels beside the decode (synthesize_many's back
        stream) hold it off; results are bit-identical either way."""
        self._pl_block += 1
        try:
            yield
        finally:
            self._pl_block -= 1

    def _pl_ok(self, st):
        """persistent layers for this state: <= PL_MAX_ROWS (<= 128) rows, a 256-CU device with room for one
        workgroup per CU, not held off, and no other lane of this engine decoding concurrently (two
        persistent grids could each hold part of the CUs)"""
        cap = self.PL_MAX_BEAM_ROWS if st.get("kv_rows") is not None else self.PL_MAX_ROWS
        return (self.pl_active and st["B"] <= min(cap, 128) and not st.get("multi_lane", False)
                and bool(self.lib.itts_gpt_pl_supported(ctypes.byref(self._cweights), st["B"])))

    def pl_takes(self, rows: int, beams: bool = False) -> bool:
        """would a decode of ``rows`` rows (beam states: utterances x num_beams) run on the persistent layers
        (no lane split, within the row cap, supported on this device)"""
        cap = self.PL_MAX_BEAM_ROWS if beams else self.PL_MAX_ROWS
        if not (self.pl_active and 0 < rows <= min(cap, 128)):
            return False
        if not beams and len(self._lane_bounds(rows, None)) > 1:
            return False
        return bool(self.lib.itts_gpt_pl_supported(ctypes.byref(self._cweights), rows))

    def pl_error(self):
        """hand-off timeout code recorded by the persistent layers (0 = none); syncs the stream."""
        if not self.pl:
            return 0
        code = ctypes.c_int(0)
        _hip.check(self.lib.itts_gpt_pl_error(self._pl_scratch.data_ptr(), _hip.stream_ptr(), ctypes.byref(code)),
                   "itts_gpt_pl_error")
        return int(code.value)

    PL_MAX_STRIKES = 3

    def _pl_recover(self, code):
        """after a hand-off timeout (some workgroup could not be placed: another grid held CUs): re-arm the
        scratch; the caller re-runs the call on the launch chain.  PL_MAX_STRIKES timeouts switch the
        persistent path off for this engine."""
        _hip.check(self.lib.itts_gpt_pl_reset(self._pl_scratch.data_ptr(), _hip.stream_ptr()), "itts_gpt_pl_reset")
        self._pl_strikes += 1
        off = self._pl_strikes >= self.PL_MAX_STRIKES
        warnings.warn(f"persistent decode layer: hand-off timeout (code {code}); re-running this call on the launch "
                      f"chain{' and keeping it off from now on' if off else ''} (results are identical)",
                      RuntimeWarning, stacklevel=3)
        if off:
            self.pl = False

    TRACES = ("step_events", "logits_trace", "beam_lineage", "beam_trace")

    def _with_pl_fallback(self, fn, *args, **kw):
        self._pl_ran = False
        # the instrumentation lists' lengths: a re-run replaces what the failed attempt recorded
        marks = {k: len(getattr(self, k)) for k in self.TRACES if getattr(self, k) is not None}
        out = fn(*args, **kw)
        if self._pl_ran:
            code = self.pl_error()
            if code:
                self._pl_recover(code)
                for k, n in marks.items():
                    del getattr(self, k)[n:]
                with self.launch_chain():
                    out = fn(*args, **kw)
        return out

    def _decode_step_fold(self, st, min_new, penalty):
        """bf16 product decode step, five launches per layer: c_attn (ln_1 folded) -> attention ->
        attn.c_proj (x += ., x^ = bf16 x) -> c_fc (ln_2 folded, gelu) -> mlp.c_proj (split-K partials +
        reduce, or full-K residual epilogue).  h holds x^ (the bf16 residual), never a LayerNorm output,
        except after the last layer, whose reduce applies ln_f + final_norm (Q5) for mel_head."""
        B, D = st["B"], self.D
        stream = _hip.stream_ptr()
        x, h, o, f = st["x"], st["h"], st["o"], st["f"]
        qkv = st["qkv"][: B * 3 * D].view(B, 3 * D)
        for li, ly in enumerate(self.layers):
            self._dgx(h, ly.wx["qkv"], B, qkv)
            kc, vc = st["kc"][li], st["vc"][li]
            rows = st.get("kv_rows")
            if rows is not None:
                _hip.check(self.lib.itts_attn_decode_rows(
                    qkv.data_ptr(), 3 * D, 1, B * 3 * D, None, kc.data_ptr(), vc.data_ptr(), kc.stride(0),
                    kc.stride(1), self.max_kv, st["pad"].data_ptr(), st["s"] + 1, st["t"].data_ptr(), o.data_ptr(), D,
                    B, self.H, _hip.dtype_code(kc), _hip.dtype_code(o), rows.data_ptr(), rows.stride(0), stream),
                    "itts_attn_decode_rows")
            else:
                _hip.check(self.lib.itts_attn_decode(
                    qkv.data_ptr(), 3 * D, 1, B * 3 * D, None, kc.data_ptr(), vc.data_ptr(), kc.stride(0),
                    kc.stride(1), self.max_kv, st["pad"].data_ptr(), st["s"] + 1, st["t"].data_ptr(), o.data_ptr(), D,
                    B, self.H, _hip.dtype_code(kc), _hip.dtype_code(o), stream), "itts_attn_decode")
            # attn.c_proj: split-K 8 partials (head pairs) + reduce (gpt_step.hip / gpt_layer.hip arithmetic)
            self._dg(o, ly.w["o"], B, None, st["ws"], epi=2, ksplit=8)
            self._reduce(st, 8, ly.b["o"], (None, None))
            self._dgx(h, ly.wx["fc"], B, f, gelu=True)
            last = li + 1 == self.L
            if self.proj_fullk and not last:
                self._dgx(f, ly.wx["proj"], B, x, epi=1, xh=h, nwaves=16)
            else:
                kp = self._ksplit(ly.w["proj"]["K"], self.KSPLIT["proj"])
                self._dg(f, ly.w["proj"], B, None, st["ws"], epi=2, ksplit=kp)
                if last:
                    self._reduce(st, kp, ly.b["proj"], self.ln_f, self.final_norm)
                else:
                    self._reduce(st, kp, ly.b["proj"], (None, None))
        self._dgw(h, self.head_w, B, self.head_b, st["logits"])
        if "kv_rows" in st:
            self._beam_step(st, 1)
        else:
            self._sample(st, 1, min_new, penalty)
        _hip.check(self.lib.itts_step_advance(st["t"].data_ptr(), 1, stream), "itts_step_advance")

    def _decode_step(self, st, min_new, penalty):
        """One fed token per row -> next token sampled (all device-side; graph-capturable)."""
        if self.cstep:
            return self._decode_step_c(st, min_new, penalty)
        if self.fold:
            return self._decode_step_fold(st, min_new, penalty)
        B, D = st["B"], self.D
        stream = _hip.stream_ptr()
        x, h, qkv, o, f = st["x"], st["h"], st["qkv"], st["o"], st["f"]
        for li, ly in enumerate(self.layers):
            if self.mode == "f32":
                self._gemm(h[:B], ly.w["qkv"], qkv[: B * 3 * D].view(B, 3 * D), bias=ly.b["qkv"])
                kq, qkv_bias = 1, None
            else:  # h = ln_1(x) was produced by the previous reduce (or the sampler for layer 0);
                # c_attn as split-K slabs, summed (+ bias) by the attention kernel
                kq, qkv_bias = self._ksplit(ly.w["qkv"]["K"], self.KSPLIT["qkv"]), ly.b["qkv"]
                self._dg(h, ly.w["qkv"], B, None, qkv, epi=2, ksplit=kq)
            kc, vc = st["kc"][li], st["vc"][li]
            if self.fuse_o:  # attention + attn.c_proj: one f32 partial per head into ws
                rows = st.get("kv_rows")
                _hip.check(self.lib.itts_attn_decode_proj(
                    qkv.data_ptr(), 3 * D, kq, B * 3 * D, _hip.ptr(qkv_bias), kc.data_ptr(), vc.data_ptr(),
                    kc.stride(0), kc.stride(1), self.max_kv, st["pad"].data_ptr(), st["s"] + 1, st["t"].data_ptr(),
                    ly.wo_io.data_ptr(), D, st["ws"].data_ptr(), B * D, D, B, self.H, _hip.dtype_code(kc),
                    _hip.ptr(rows), 0 if rows is None else rows.stride(0), stream), "itts_attn_decode_proj")
            elif "kv_rows" in st:  # beams: keys read through the lineage table
                _hip.check(self.lib.itts_attn_decode_rows(
                    qkv.data_ptr(), 3 * D, kq, B * 3 * D, _hip.ptr(qkv_bias), kc.data_ptr(), vc.data_ptr(),
                    kc.stride(0), kc.stride(1), self.max_kv, st["pad"].data_ptr(), st["s"] + 1, st["t"].data_ptr(),
                    o.data_ptr(), D, B, self.H, _hip.dtype_code(kc), _hip.dtype_code(o), st["kv_rows"].data_ptr(),
                    st["kv_rows"].stride(0), stream), "itts_attn_decode_rows")
            else:
                _hip.check(self.lib.itts_attn_decode(
                    qkv.data_ptr(), 3 * D, kq, B * 3 * D, _hip.ptr(qkv_bias), kc.data_ptr(), vc.data_ptr(),
                    kc.stride(0), kc.stride(1), self.max_kv, st["pad"].data_ptr(), st["s"] + 1, st["t"].data_ptr(),
                    o.data_ptr(), D, B, self.H, _hip.dtype_code(kc), _hip.dtype_code(o), stream), "itts_attn_decode")
            nxt = self.layers[li + 1].ln1 if li + 1 < self.L else None
            if self.mode == "f32":
                self._gemm(o[:B], ly.w["o"], x, bias=ly.b["o"], residual=True)
                self._ln(x, h, ly.ln2, M=B)
                self._gemm(h[:B], ly.w["fc"], f, bias=ly.b["fc"], gelu=True)
                self._gemm(f[:B], ly.w["proj"], x, bias=ly.b["proj"], residual=True)
                if nxt is not None:
                    self._ln(x, h, nxt, M=B)
                else:
                    self._ln(x, h, self.ln_f, self.final_norm, M=B)
                continue
            if self.fuse_o:
                self._reduce(st, self.H, ly.b["o"], ly.ln2)
            else:
                ko = self._ksplit(ly.w["o"]["K"], self.KSPLIT["o"])
                self._dg(o, ly.w["o"], B, None, st["ws"], epi=2, ksplit=ko)
                self._reduce(st, ko, ly.b["o"], ly.ln2)
            self._dgw(h, ly.w["fc"], B, ly.b["fc"], f, gelu=True)
            kp = self._ksplit(ly.w["proj"]["K"], self.KSPLIT["proj"])
            self._dg(f, ly.w["proj"], B, None, st["ws"], epi=2, ksplit=kp)
            if nxt is not None:
                self._reduce(st, kp, ly.b["proj"], nxt)
            else:
                self._reduce(st, kp, ly.b["proj"], self.ln_f, self.final_norm)
        if self.mode == "f32":
            self._gemm(h[:B], self.head_w, st["logits"], bias=self.head_b)
        else:
            self._dgw(h, self.head_w, B, self.head_b, st["logits"])
        if "kv_rows" in st:
            self._beam_step(st, 1)
        else:
            self._sample(st, 1, min_new, penalty)
        _hip.check(self.lib.itts_step_advance(st["t"].data_ptr(), 1, stream), "itts_step_advance")

    # split-K factors of the residual projections (partials reduced by itts_residual_reduce_ln);
    # ITTS_KSPLIT="qkv,o,proj" overrides them (tuning sweeps)
    KSPLIT = {"qkv": 2, "o": 8, "proj": 8}  # "o" 2 -> 8: 864 -> 849 us per step (sweep, round 1)
    if os.environ.get("ITTS_KSPLIT"):
        KSPLIT = dict(zip(("qkv", "o", "proj"), (int(v) for v in os.environ["ITTS_KSPLIT"].split(","))))

    @staticmethod
    def _ksplit(K, want):
        ks = want
        while ks > 1 and (K // 16) % ks:
            ks //= 2
        return ks

    def _dgw(self, A, w, M, bias, Y, gelu=False):
        """store-epilogue projection (c_fc + gelu, mel_head): 16-column tiles when packed for them."""
        if "sk16" not in w:
            return self._dg(A, w, M, bias, Y, gelu=gelu)
        _hip.check(self.lib.itts_decode_gemm16(
            A.data_ptr(), A.stride(0), w["sk16"].data_ptr(), w["K"], w["N"], M, _hip.ptr(bias), int(gelu),
            Y.data_ptr(), Y.stride(0), _hip.dtype_code(Y), _hip.stream_ptr()), "itts_decode_gemm16")

    def _dg(self, A, w, M, bias, Y, ln=None, ln2=None, gelu=False, epi=0, ksplit=1):
        """itts_decode_gemm: Y = act(prologue(A) @ W^T + bias) (epi 0), Y += ... (epi 1), or split-K
        partial products into Y (epi 2); the prologue is identity (bf16 A) or the (double) LayerNorm of
        the f32 residual stream A."""
        mode = 0 if ln is None else (1 if ln2 is None else 2)
        N = w["N"]
        _hip.check(self.lib.itts_decode_gemm(
            A.data_ptr(), A.stride(0), w["sk"].data_ptr(), w["K"], N, M, _hip.ptr(bias),
            None if ln is None else ln[0].data_ptr(), None if ln is None else ln[1].data_ptr(),
            None if ln2 is None else ln2[0].data_ptr(), None if ln2 is None else ln2[1].data_ptr(),
            mode, int(gelu), epi, Y.data_ptr(), N if epi == 2 else Y.stride(0), _hip.dtype_code(Y),
            M * N, ksplit, _hip.stream_ptr()), "itts_decode_gemm")

    def _reduce(self, st, nsplit, bias, ln, ln2=None):
        """x += bias + sum of the split-K partials (fixed order); h = LN(x) (or LN2(LN(x)))."""
        B, D = st["B"], self.D
        x, h = st["x"], st["h"]
        _hip.check(self.lib.itts_residual_reduce_ln(
            x.data_ptr(), D, st["ws"].data_ptr(), nsplit, B * D, D, bias.data_ptr(), h.data_ptr(), D, B, D,
            _hip.ptr(ln[0]), _hip.ptr(ln[1]), None if ln2 is None else ln2[0].data_ptr(),
            None if ln2 is None else ln2[1].data_ptr(), _hip.dtype_code(h), _hip.stream_ptr()),
            "itts_residual_reduce_ln")

    # ---------------- public: generate ----------------
    # Row chunks ("lanes") decode concurrently, each on its own HIP stream with its own captured
    # graph and state: one decode step is a chain of ~150 small dependent kernels (latency-bound at
    # batch 32), so two independent chains keep more of the GPU busy; the second lane re-reads each
    # layer's weights shortly after the first, out of the 256 MiB Infinity Cache.  Rows never
    # interact, so the ids do not depend on the lane split.
    LANES = 1  # measured: 2 lanes of 16 rows are slower than 1 lane of 32 (half-size steps cost nearly as much)
    MIN_LANE_ROWS = 8

    def _lane_bounds(self, B: int, lanes: Optional[int]):
        n = self.LANES if lanes is None else max(1, int(lanes))
        n = max(1, min(n, B // self.MIN_LANE_ROWS)) if lanes is None else min(n, B)
        step = (B + n - 1) // n
        return [(r, min(B, r + step)) for r in range(0, B, step)]

    MAX_CACHED_SHAPES = 4  # decode states (+ captured graphs) kept per lane, LRU

    def _lane(self, i: int, rows: int, max_new: int, s: int):
        """decode state + captured graph for lane i at this (rows, max_new, prompt length) shape; a few
        shapes stay cached so that alternating bucket shapes (long-form driver) do not re-capture."""
        lanes = self.__dict__.setdefault("_lanes", {})
        key = (rows, max_new, s)
        ln = lanes.pop((i, key), None)
        if ln is None:
            mine = [k for k in lanes if isinstance(k, tuple) and len(k) == 2 and k[0] == i and isinstance(k[1], tuple)]
            if len(mine) >= self.MAX_CACHED_SHAPES:  # evict the least recently used shape first
                del lanes[mine[0]]
                torch.cuda.empty_cache()
            ln = {"key": key, "st": self._alloc_state(rows, max_new), "graph": None,
                  "stream": lanes.get(("stream", i)) or torch.cuda.Stream(self.dev)}
            lanes[("stream", i)] = ln["stream"]
        lanes[(i, key)] = ln  # (re)inserted last = most recently used
        return ln

    @torch.no_grad()
    def generate(self, conds: torch.Tensor, text_ids: torch.Tensor, max_new_tokens: int,
                 repetition_penalty: float = 10.0, min_new_tokens: int = 0, use_graph: bool = True,
                 check_every: int = 16, forced_codes: Optional[torch.Tensor] = None, do_sample: bool = False,
                 temperature: float = 1.0, top_k: int = 0, top_p: float = 1.0,
                 seed: Optional[int] = None, lanes: Optional[int] = None, num_beams: int = 1,
                 length_penalty: float = 0.0) -> torch.Tensor:
        """Greedy (do_sample=False) or top-k/top-p sampling (do_sample=True; num_beams=1) decode
        -> codes [B, n] int64 on the device, finished rows padded with the stop token, n = steps until
        every row stopped (or max_new_tokens).  ``seed`` (default: drawn from torch's CPU generator)
        keys the device RNG (by global row), so a fixed seed reproduces the draws for any lane split.
        num_beams > 1: beam search / beam sample (``generate_beam``)."""
        if num_beams and num_beams > 1:
            assert forced_codes is None, "teacher forcing is a num_beams=1 test feature"
            return self.generate_beam(conds, text_ids, max_new_tokens, num_beams, repetition_penalty,
                                      length_penalty, min_new_tokens, do_sample, temperature, top_k, top_p, seed,
                                      use_graph, check_every)
        if do_sample and seed is None:  # drawn once: a re-run on the launch chain makes the same draws
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        return self._with_pl_fallback(self._generate, conds, text_ids, max_new_tokens, repetition_penalty,
                                      min_new_tokens, use_graph, check_every, forced_codes, do_sample, temperature,
                                      top_k, top_p, seed, lanes)

    def _generate(self, conds, text_ids, max_new_tokens, repetition_penalty, min_new_tokens, use_graph, check_every,
                  forced_codes, do_sample, temperature, top_k, top_p, seed, lanes):
        emb, pad, s = self.prepare_inputs(conds, text_ids)
        B = emb.shape[0]
        assert s + 1 + max_new_tokens <= self.max_kv, "KV capacity exceeded"
        sampling = (float(temperature), int(top_k), float(top_p)) if do_sample else None
        gkey = (min_new_tokens, repetition_penalty, sampling, forced_codes is not None, self.cstep, self.pl_active)
        main = torch.cuda.current_stream(self.dev)
        work = []
        bounds = self._lane_bounds(B, lanes)
        for i, (r0, r1) in enumerate(bounds):
            ln = self._lane(i, r1 - r0, max_new_tokens, s)
            if ln["st"].get("multi_lane", False) != (len(bounds) > 1):
                ln["st"]["multi_lane"] = len(bounds) > 1
                self._drop_graphs(ln)  # captured for the other decode path
            ln["stream"].wait_stream(main)  # inputs prepared on the caller's stream
            with torch.cuda.stream(ln["stream"]):
                self._start_lane(ln, emb[r0:r1], pad[r0:r1], s, r0, sampling, seed,
                                 None if forced_codes is None else forced_codes[r0:r1], min_new_tokens,
                                 repetition_penalty, use_graph and max_new_tokens > 1, gkey)
            work.append(ln)
        self._pl_ran = any(self._pl_ok(ln["st"]) for ln in work)
        steps = 1
        trace = self.logits_trace  # optional instrumentation (tests): raw f32 logits of every step
        assert trace is None or len(work) == 1, "logits tracing needs a single lane"
        ev = self.step_events  # optional instrumentation: HIP events around each lane's step
        keys0 = [int((r1 - r0) * (s + 2)) - int(pad[r0:r1].sum()) for r0, r1 in self._lane_bounds(B, lanes)] \
            if ev is not None else None
        kmulti = self.GRAPH_STEPS if (len(work) == 1 and trace is None and work[0]["graph_ok"]) else 1
        while steps < max_new_tokens:
            # kmulti decode steps per graph replay (one captured graph holds kmulti steps) while whole
            # groups fit before max_new_tokens and inside one done-check interval
            n = kmulti if (kmulti > 1 and steps + kmulti <= max_new_tokens
                           and (steps % check_every) + kmulti <= check_every) else 1
            for li, ln in enumerate(work):
                with torch.cuda.stream(ln["stream"]):
                    if ev is not None:
                        e0 = torch.cuda.Event(enable_timing=True)
                        e0.record()
                    if n > 1:
                        self._multi_graph(ln, n, min_new_tokens, repetition_penalty, gkey).replay()
                    elif ln["graph_ok"]:
                        ln["graph"][0].replay()
                    else:
                        self._decode_step(ln["st"], min_new_tokens, repetition_penalty)
                    if ev is not None:
                        e1 = torch.cuda.Event(enable_timing=True)
                        e1.record()
                        # keys attended per step, summed over the lane's rows: s + 2 + r - pad_b (a
                        # multi-step replay: its interval once, then zero-length entries per extra step)
                        for j in range(n):
                            ev.append((e0 if j == 0 else e1, e1, ln["st"]["B"],
                                       keys0[li] + ln["st"]["B"] * (steps - 1 + j)))
                    if trace is not None:
                        trace.append(ln["st"]["logits"][:, : self.V].clone())
            prev = steps
            steps += n
            if steps // check_every != prev // check_every:
                done = True
                for ln in work:
                    with torch.cuda.stream(ln["stream"]):
                        done = done and bool(ln["st"]["done"].all())
                if done:
                    break
        for ln in work:
            main.wait_stream(ln["stream"])
        codes = torch.cat([ln["st"]["codes"][:, :steps] for ln in work], 0).long()
        hit = codes == self.stop_mel
        if bool(hit.any(dim=1).all()):
            n = int(hit.int().argmax(dim=1).max()) + 1
            codes = codes[:, :n]
        return codes

    def _start_lane(self, ln, emb, pad, s, row0, sampling, seed, forced, min_new, penalty, use_graph, gkey):
        """reset one lane's decode state, run its prefill + first token, (re)capture its graph."""
        st = ln["st"]
        B = st["B"]
        st["s"] = s
        st["pad"].copy_(pad)  # never rebind: the captured graph holds this pointer
        st["seen"].zero_()
        st["seen"][:, 1] = 1
        st["seen"][:, self.start_mel] = 1
        st["done"].zero_()
        st["codes"].fill_(self.stop_mel)
        st["sampling"] = sampling
        sd = [0, 0] if seed is None else [(seed >> 32 * i) & 0xFFFFFFFF for i in range(2)]
        sd = [v - (1 << 32) if v >= 1 << 31 else v for v in sd]
        st["t"].copy_(torch.tensor([0, row0, sd[0], sd[1]], dtype=torch.int32))
        if forced is not None:  # teacher forcing (tests): feed these ids, record the chosen ids
            fc = torch.full((B, st["max_new"]), self.stop_mel, dtype=torch.int32, device=self.dev)
            fc[:, : forced.shape[1]] = forced.to(self.dev, torch.int32)
            if st.get("forced") is None:
                st["forced"] = fc
                self._drop_graphs(ln)  # every graph holds the forced-codes pointer
            else:
                st["forced"].copy_(fc)
        elif st.get("forced") is not None:
            st["forced"] = None
            self._drop_graphs(ln)
        # ---- prefill over [B, s+1] rows ----
        M = B * (s + 1)
        x = emb.reshape(M, self.D).contiguous()
        starts = torch.arange(B, dtype=torch.int32, device=self.dev) * (s + 1)
        lens = torch.full((B,), s + 1, dtype=torch.int32, device=self.dev)
        last = (starts + s).contiguous()
        if self.cseq and (self.fold or self.mode == "f32") and "kv_rows" not in st:
            # one C-ABI call: layers -> KV cache, head, first token + next embedding (itts_gpt_prefill)
            st["s"] = s
            smp = st.get("sampling")
            mode = _hip.Sampling(0, int(min_new), float(penalty), 1.0, 0, 1.0) if smp is None else \
                _hip.Sampling(1, int(min_new), float(penalty), float(smp[0]), int(smp[1]), float(smp[2]))
            ws = self._seq_workspace(M)
            _hip.check(self.lib.itts_gpt_prefill(
                ctypes.byref(self._c_seq_weights()), ctypes.byref(self._c_head_weights()),
                ctypes.byref(self._c_state(st)), x.data_ptr(), s, starts.data_ptr(), lens.data_ptr(), last.data_ptr(),
                ctypes.byref(mode), ws.data_ptr(), _hip.stream_ptr()), "itts_gpt_prefill")
            self._after_prefill(ln, st, min_new, penalty, use_graph, gkey)
            return
        self._forward_rows(x, starts, lens, pad, s + 1, cache=(st["kc"], st["vc"]))
        self._ln(x, st["h"], self.ln_f, self.final_norm, idx=last, M=B)
        if self.mode == "f32":
            self._gemm(st["h"][:B], self.head_w, st["logits"], bias=self.head_b)
        else:
            self._dgw(st["h"], self.head_w, B, self.head_b, st["logits"])
        self._sample(st, 0, min_new, penalty)
        self._after_prefill(ln, st, min_new, penalty, use_graph, gkey)

    def _after_prefill(self, ln, st, min_new, penalty, use_graph, gkey):
        if self.logits_trace is not None:  # the prefill's logits (before the capture's warm-up step)
            self.logits_trace.append(st["logits"][:, : self.V].clone())
        ln["graph_ok"] = False
        if use_graph:
            ln["graph"] = (self._cached_graph(ln, gkey, lambda: self._capture(st, min_new, penalty)), gkey)
            ln["graph_ok"] = True

    # captured graphs kept per lane, keyed by what they were captured for (one-step and multi-step graphs of the
    # persistent layers and of the launch chain): synthesize_many's overlap alternates between the two decode paths
    # for the same shape, which recaptured at every switch with one slot per lane
    GRAPH_CACHE = 4

    def _keep_graph(self, ln, key, g):
        cache = ln.setdefault("graphs", {})
        cache.pop(key, None)
        cache[key] = g
        while len(cache) > self.GRAPH_CACHE:
            cache.pop(next(iter(cache)))  # oldest first

    def _cached_graph(self, ln, gkey, capture):
        cache = ln.setdefault("graphs", {})
        g = cache.get(("one", gkey))
        if g is None:
            g = capture()
        self._keep_graph(ln, ("one", gkey), g)
        return g

    @staticmethod
    def _drop_graphs(ln):
        ln["graph"] = ln["multi"] = None
        ln["graphs"] = {}

    MUTABLE = ("t", "x", "h", "seen", "done", "codes")
    BEAM_MUTABLE = ("beam_score", "kv_rows", "done_u", "hyp_score", "hyp_len", "hyp_codes", "hyp_n", "hyp_order",
                    "hyp_worst")

    # decode steps per captured graph replay (ITTS_GRAPH_STEPS; 1 = one step per replay): 4 steps
    # per graph 776 vs 785 us per step (profiles/graph_steps_r02.txt: the boundary between two graph
    # launches costs more than a kernel boundary inside one graph)
    # round 4, persistent layers: 4 / 8 / 16 steps per replay 661.6 / 659.2 / 659.9 us per C3 step
    # (profiles/env_ab2.sh, two interleaved reps each)
    GRAPH_STEPS = int(os.environ.get("ITTS_GRAPH_STEPS", "8"))

    def _multi_graph(self, ln, n, min_new, penalty, gkey):
        """the lane's n-step graph (captured on first use, like the one-step graph)."""
        mg = ln.get("multi")
        if mg is not None and mg[1] == (n, gkey):
            return mg[0]
        cached = ln.setdefault("graphs", {}).get(("multi", n, gkey))
        if cached is not None:
            ln["multi"] = (cached, (n, gkey))
            return cached
        st = ln["st"]
        keys = self.MUTABLE + (self.BEAM_MUTABLE if "kv_rows" in st else ())
        saved = {k: st[k].clone() for k in keys}
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            if self.cstep and "kv_rows" not in st:  # n steps, one counter advance
                self._decode_step_c(st, min_new, penalty, nsteps=n)
            else:
                for _ in range(n):
                    self._decode_step(st, min_new, penalty)
        for k, v in saved.items():
            st[k].copy_(v)
        self._keep_graph(ln, ("multi", n, gkey), g)
        ln["multi"] = (g, (n, gkey))
        return g

    def _capture(self, st, min_new, penalty):
        """Capture one decode step into a hipGraph; counters are device-side so replays advance."""
        keys = self.MUTABLE + (self.BEAM_MUTABLE if "kv_rows" in st else ())
        saved = {k: st[k].clone() for k in keys}
        cur = torch.cuda.current_stream(self.dev)
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            self._decode_step(st, min_new, penalty)  # warm-up (also validates launches)
        cur.wait_stream(s)
        for k, v in saved.items():  # restore the state mutated by the warm-up step
            st[k].copy_(v)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._decode_step(st, min_new, penalty)
        return g  # capture does not execute the kernels; state is intact

    # ---------------- beam search / beam sample (num_beams > 1) ----------------
    def _beam_step(self, st, col_delta):
        """candidates per row, then per-utterance selection + reorder + next embedding (gpt_beam.hip)."""
        bm = st["beam"]
        stream = _hip.stream_ptr()
        R, K = st["B"], bm["K"]
        smp = bm["sampling"]
        _hip.check(self.lib.itts_beam_candidates(
            st["logits"].data_ptr(), self.Vp, self.V, st["seen"].data_ptr(), st["beam_score"].data_ptr(),
            st["t"].data_ptr(), col_delta, int(bm["min_new"]), self.stop_mel, float(bm["penalty"]), int(smp is not None),
            float(smp[0]) if smp else 1.0, int(smp[1]) if smp else 0, float(smp[2]) if smp else 1.0, K,
            st["cand_key"].data_ptr(), st["cand_score"].data_ptr(), st["cand_tok"].data_ptr(), R, stream),
            "itts_beam_candidates")
        ln1 = self._embed_ln()
        _hip.check(self.lib.itts_beam_select(
            st["cand_key"].data_ptr(), st["cand_score"].data_ptr(), st["cand_tok"].data_ptr(), K, self.V,
            self.stop_mel, int(smp is not None), float(bm["length_penalty"]), st["t"].data_ptr(), col_delta,
            st["done_u"].data_ptr(), st["beam_score"].data_ptr(), st["codes"].data_ptr(), st["max_new"],
            st["seen"].data_ptr(), self.Vp, st["base_ids"].data_ptr(), st["base_ids"].numel(),
            st["kv_rows"].data_ptr(), st["kv_rows"].stride(0), st["s"] + 1, st["hyp_score"].data_ptr(),
            st["hyp_len"].data_ptr(), st["hyp_codes"].data_ptr(), st["hyp_n"].data_ptr(), st["hyp_order"].data_ptr(),
            st["hyp_worst"].data_ptr(), self.mel_emb.data_ptr(), self.mel_pos.data_ptr(), 2, self.D,
            ln1[0], ln1[1], st["x"].data_ptr(), st["h"].data_ptr(), _hip.dtype_code(st["h"]),
            R // K, st["max_new"], stream), "itts_beam_select")

    def _beam_state(self, B: int, K: int, max_new: int, s: int):
        key = ("beam", B, K, max_new, s)
        ln = self._lanes.get("beam")
        if ln is None or ln["key"] != key:
            if ln is not None:
                self._lanes.pop("beam")
                del ln
                torch.cuda.empty_cache()
            R = B * K
            st = self._alloc_state(R, max_new)
            dev = self.dev
            st.update({
                "beam_score": torch.zeros(R, device=dev),
                "cand_key": torch.zeros(R, 2 * K, device=dev),
                "cand_score": torch.zeros(R, 2 * K, device=dev),
                "cand_tok": torch.zeros(R, 2 * K, dtype=torch.int32, device=dev),
                "kv_rows": torch.zeros(R, self.max_kv, dtype=torch.int32, device=dev),
                "done_u": torch.zeros(B, dtype=torch.uint8, device=dev),
                "hyp_score": torch.zeros(B, K, device=dev),
                "hyp_len": torch.zeros(B, K, dtype=torch.int32, device=dev),
                "hyp_codes": torch.zeros(B, K, max_new, dtype=torch.int32, device=dev),
                "hyp_n": torch.zeros(B, dtype=torch.int32, device=dev),
                "hyp_order": torch.zeros(B, K, dtype=torch.int32, device=dev),
                "hyp_worst": torch.zeros(B, device=dev),
                "base_ids": torch.tensor([1, self.start_mel], dtype=torch.int32, device=dev),
            })
            ln = {"key": key, "st": st, "graph": None}
            self._lanes["beam"] = ln
        return ln

    @torch.no_grad()
    def generate_beam(self, conds: torch.Tensor, text_ids: torch.Tensor, max_new_tokens: int, num_beams: int = 3,
                      repetition_penalty: float = 10.0, length_penalty: float = 0.0, min_new_tokens: int = 0,
                      do_sample: bool = False, temperature: float = 1.0, top_k: int = 0, top_p: float = 1.0,
                      seed: Optional[int] = None, use_graph: bool = True, check_every: int = 16) -> torch.Tensor:
        """``generate(num_beams=K)`` of inference_speech (gpt/model.py:698-703) with transformers 4.36
        ``beam_search`` (do_sample=False) / ``beam_sample`` (do_sample=True) semantics -- the
        reference's default decoding (infer.py:535-543).  Rows r = b*K + k; the prompt is prefilled
        once per utterance (cache row b*K) and shared through the KV lineage table.
        -> codes [B, n] int64 (best hypothesis, then the stop token, padded with it)."""
        K = int(num_beams)
        assert 2 <= K <= 16, "num_beams must be in [2, 16]"
        if self.max_kv > self.BEAM_MAX_KV:  # both beam attentions stage the lineage rows of a key range in LDS
            raise ValueError(f"beam decoding supports a KV capacity of at most {self.BEAM_MAX_KV} positions "
                             f"(this engine: max_kv={self.max_kv}); build the engine with a smaller max_kv")
        if do_sample and seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        return self._with_pl_fallback(self._generate_beam, conds, text_ids, max_new_tokens, K, repetition_penalty,
                                      length_penalty, min_new_tokens, do_sample, temperature, top_k, top_p, seed,
                                      use_graph, check_every)

    def _generate_beam(self, conds, text_ids, max_new_tokens, K, repetition_penalty, length_penalty, min_new_tokens,
                       do_sample, temperature, top_k, top_p, seed, use_graph, check_every):
        emb, pad, s = self.prepare_inputs(conds, text_ids)
        B = emb.shape[0]
        R = B * K
        assert s + 1 + max_new_tokens <= self.max_kv, "KV capacity exceeded"
        sampling = (float(temperature), int(top_k), float(top_p)) if do_sample else None
        ln = self._beam_state(B, K, max_new_tokens, s)
        st = ln["st"]
        st["s"] = s
        self._pl_ran = self._pl_ok(st)
        st["beam"] = {"K": K, "sampling": sampling, "min_new": min_new_tokens, "penalty": repetition_penalty,
                      "length_penalty": length_penalty}
        rows_b = torch.arange(B, device=self.dev).repeat_interleave(K)
        st["pad"].copy_(pad[rows_b])
        st["seen"].zero_()
        st["seen"][:, 1] = 1
        st["seen"][:, self.start_mel] = 1
        st["done"].zero_()
        st["done_u"].zero_()
        st["codes"].fill_(self.stop_mel)
        bs = torch.zeros(B, K, device=self.dev)
        if not do_sample:
            bs[:, 1:] = -1e9  # HF 4.36 beam_search: only beam 0 expands at the first step
        st["beam_score"].copy_(bs.view(-1))
        st["kv_rows"].copy_((rows_b * K).int()[:, None].expand(R, self.max_kv))
        st["hyp_n"].zero_()
        st["hyp_worst"].fill_(1e9)
        sd = [0, 0] if seed is None else [(seed >> 32 * i) & 0xFFFFFFFF for i in range(2)]
        sd = [v - (1 << 32) if v >= 1 << 31 else v for v in sd]
        st["t"].copy_(torch.tensor([0, 0, sd[0], sd[1]], dtype=torch.int32))
        # ---- prefill of the B prompts into cache rows b*K ----
        M = B * (s + 1)
        x = emb.reshape(M, self.D).contiguous()
        starts = torch.arange(B, dtype=torch.int32, device=self.dev) * (s + 1)
        lens = torch.full((B,), s + 1, dtype=torch.int32, device=self.dev)
        self._forward_rows(x, starts, lens, pad, s + 1, cache=(st["kc"][:, ::K], st["vc"][:, ::K]))
        last = (starts + s)[rows_b].contiguous()
        self._ln(x, st["h"], self.ln_f, self.final_norm, idx=last, M=R)
        if self.mode == "f32":
            self._gemm(st["h"][:R], self.head_w, st["logits"], bias=self.head_b)
        else:
            self._dgw(st["h"], self.head_w, R, self.head_b, st["logits"])
        self._beam_step(st, 0)
        btr = self.beam_trace

        def trace_step(n_done):
            btr.append((st["codes"][:, :n_done].cpu(), st["beam_score"].cpu(), st["done_u"].cpu()))

        if btr is not None:
            trace_step(1)
        gkey = (K, min_new_tokens, repetition_penalty, length_penalty, sampling, self.cstep, self.pl_active)
        graph_ok = use_graph and max_new_tokens > 1
        if graph_ok and (ln["graph"] is None or ln["graph"][1] != gkey):
            ln["graph"] = (self._cached_graph(ln, gkey, lambda: self._capture(st, min_new_tokens, repetition_penalty)),
                           gkey)
        steps = 1
        ev = self.step_events  # optional instrumentation (bench.py): HIP events around each step
        # distinct cache keys a step reads: each utterance's prompt once (shared by its beams through
        # the lineage table) + every beam row's generated keys
        keys0 = int(B * (s + 1) - int(pad.sum())) if ev is not None else 0
        kmulti = self.GRAPH_STEPS if graph_ok and btr is None else 1
        while steps < max_new_tokens:
            n = kmulti if (kmulti > 1 and steps + kmulti <= max_new_tokens
                           and (steps % check_every) + kmulti <= check_every) else 1
            if ev is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            if n > 1:
                self._multi_graph(ln, n, min_new_tokens, repetition_penalty, gkey).replay()
            elif graph_ok:
                ln["graph"][0].replay()
            else:
                self._decode_step(st, min_new_tokens, repetition_penalty)
            if ev is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                if self.beam_lineage is not None:  # after the event: not inside the timed interval
                    self.beam_lineage.append((len(ev), steps, n, st["kv_rows"].clone()))
                for j in range(n):
                    ev.append((e0 if j == 0 else e1, e1, R, keys0 + R * (steps + j)))
            prev = steps
            steps += n
            if btr is not None:
                trace_step(steps)
            if steps // check_every != prev // check_every and bool(st["done_u"].all()):
                break
        if ev is not None and self.beam_lineage is not None:  # resolved by the caller, outside its timed region
            self.beam_lineage.append(("shape", B, K, s + 1, keys0))
        return self._beam_finalize(st, B, K, steps, max_new_tokens, length_penalty)

    @staticmethod
    def beam_distinct_keys(ev, lineage):
        """Rewrite each beam step's key count (ev[i][3]) as the distinct K/V rows it reads: every utterance's
        prompt once, the generated positions once per DISTINCT cache row among its beams' lineages (from the
        lineage table at the end of the step's replay), and this step's new key of every row.  ``lineage``:
        what generate_beam recorded with ``beam_lineage`` set (snapshots, then a ("shape", ...) entry per call)."""
        recs = []
        for e in lineage:
            if e[0] == "shape":
                _, B, K, kv_base, keys0 = e
                HipGPT._beam_distinct_keys_call(ev, recs, B, K, kv_base, keys0)
                recs = []
            else:
                recs.append(e)

    @staticmethod
    def _beam_distinct_keys_call(ev, lineage, B, K, kv_base, keys0):
        R = B * K
        for i0, step0, n, snap in lineage:
            kv = snap.view(B, K, -1)
            for j in range(n):
                t = step0 + j  # this step writes position kv_base + t - 1 of every row
                gen = kv[:, :, kv_base: kv_base + t - 1]
                if gen.shape[2] > 0:
                    srt = gen.sort(dim=1).values
                    distinct = int(gen.shape[0] * gen.shape[2] + (srt[:, 1:] != srt[:, :-1]).sum())
                else:
                    distinct = 0
                e0, e1, rows, _ = ev[i0 + j]
                ev[i0 + j] = (e0, e1, rows, keys0 + distinct + R)

    def _beam_finalize(self, st, B, K, steps, max_new, length_penalty):
        """BeamSearchScorer.finalize: open beams of unfinished utterances become hypotheses (generated
        length = steps); the best hypothesis per utterance, then eos, padded (HF beam_search.py)."""
        done = st["done_u"].cpu().numpy()
        hs, hl = st["hyp_score"].cpu().numpy(), st["hyp_len"].cpu().numpy()
        hc, hn, ho = st["hyp_codes"].cpu().numpy(), st["hyp_n"].cpu().numpy(), st["hyp_order"].cpu().numpy()
        hw = st["hyp_worst"].cpu().numpy()
        codes = st["codes"][:, :steps].cpu().numpy()
        scores = st["beam_score"].cpu().numpy()
        best = []
        for b in range(B):
            hyps = [(float(hs[b, ho[b, i]]), list(hc[b, ho[b, i], : hl[b, ho[b, i]]])) for i in range(hn[b])]
            worst = float(hw[b])
            if not done[b]:
                for k in range(K):
                    sc = float(scores[b * K + k]) / (steps ** length_penalty)
                    if len(hyps) < K or sc > worst:
                        hyps.append((sc, list(codes[b * K + k])))
                        if len(hyps) > K:
                            order = sorted((h[0], i) for i, h in enumerate(hyps))
                            del hyps[order[0][1]]
                            worst = order[1][0]
                        else:
                            worst = min(sc, worst)
            best.append(sorted(hyps, key=lambda h: h[0])[-1][1])
        n = min(max(len(t) for t in best) + 1, max_new)
        out = torch.full((B, n), self.stop_mel, dtype=torch.long)
        for b, t in enumerate(best):
            out[b, : len(t)] = torch.tensor(t, dtype=torch.long)
        return out.to(self.dev)

    # ---------------- latent pass ----------------
    @torch.no_grad()
    def latent(self, conds: torch.Tensor, text_list: List[torch.Tensor], codes_list: List[torch.Tensor]):
        """Teacher-forced pass for each utterance (gpt/model.py:521-578, return_latent=True).

        conds [B|1, 32, D]; text_list[b] = ids [L_b] (used as given); codes_list[b] = codes [n_b]
        -> (latent [B, Tmax, D] in the vocoder's input layout (bf16 in bf16 mode), lengths [B])."""
        B = len(text_list)
        conds = conds.to(self.dev).float()
        ncond, D, dev = conds.shape[1], self.D, self.dev
        # all index arithmetic on the host (one copy of the text ids down, one of each index up), then
        # three gathers build the packed [M, D] input: [conds ; text_emb + text_pos ; mel_emb + mel_pos]
        t_host = [t.reshape(-1) for t in text_list]
        t_all = torch.cat([t.to(dev) for t in t_host]).long().cpu().numpy() if B else np.zeros(0, np.int64)
        lt = np.array([t.numel() for t in t_host], dtype=np.int64)
        codes_np = [np.asarray(c.reshape(-1).cpu(), dtype=np.int64) for c in codes_list]
        n = [int(c.shape[0]) for c in codes_np]
        lens = (ncond + lt + 2 + np.array(n, dtype=np.int64) + 2).tolist()
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        M = int(sum(lens))
        cond_dst, cond_src, txt_dst, txt_tok, txt_pos, mel_dst, mel_tok, mel_pos = ([] for _ in range(8))
        toff = np.concatenate([[0], np.cumsum(lt)[:-1]]).astype(np.int64)
        for b in range(B):
            s0 = int(starts[b])
            cond_dst.append(np.arange(s0, s0 + ncond))
            cond_src.append((0 if conds.shape[0] == 1 else b) * ncond + np.arange(ncond))
            tt = np.concatenate([[self.start_text], t_all[toff[b]: toff[b] + lt[b]], [self.stop_text]])
            txt_dst.append(s0 + ncond + np.arange(tt.shape[0]))
            txt_tok.append(tt)
            txt_pos.append(np.arange(tt.shape[0]))
            mm = np.concatenate([[self.start_mel], codes_np[b], [self.stop_mel]])
            m0 = s0 + ncond + tt.shape[0]
            mel_dst.append(m0 + np.arange(mm.shape[0]))
            mel_tok.append(mm)
            mel_pos.append(np.arange(mm.shape[0]))
        up = lambda parts: torch.from_numpy(np.concatenate(parts).astype(np.int64)).to(dev)  # noqa: E731
        x = torch.empty(M, D, device=dev)
        x[up(cond_dst)] = conds.reshape(-1, D)[up(cond_src)]
        x[up(txt_dst)] = self.text_emb[up(txt_tok)] + self.text_pos[up(txt_pos)]
        x[up(mel_dst)] = self.mel_emb[up(mel_tok)] + self.mel_pos[up(mel_pos)]
        s_t = torch.from_numpy(starts.astype(np.int32)).to(dev)
        l_t = torch.tensor(lens, dtype=torch.int32, device=dev)
        Tmax = max(n)
        idx = np.zeros((B, Tmax), dtype=np.int32)
        for b in range(B):  # latent rows: the first n of the mel block (start token .. code n-2), :-2 of
            first = int(starts[b]) + ncond + int(lt[b]) + 2  # gpt/model.py:575-578
            idx[b, : n[b]] = np.arange(first, first + n[b])
        out = torch.empty(B, Tmax, self.D, dtype=self.act_dtype, device=self.dev)
        self._forward_rows(x, s_t, l_t, None, max(lens), out_idx=torch.from_numpy(idx).to(dev).view(-1), out=out)
        return out, torch.tensor(n, dtype=torch.int32)


F32, BF16 = _hip.F32, _hip.BF16
