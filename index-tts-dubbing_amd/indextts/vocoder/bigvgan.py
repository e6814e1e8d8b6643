"""BigVGAN2 vocoder on the HIP C-ABI (speech-code latents -> 24 kHz waveform).

Mirrors ``BigVGAN.forward`` (reference ``indextts/BigVGAN/models.py:201-250``) for a whole batch of
utterances at once, with per-utterance lengths (ragged batches are exact: every conv and
activation clamps/zero-pads at each utterance's own edges, as if it ran alone at batch 1 like the
reference's ``infer()``).

HBM layout: channel-last ``[B, T_stage, C]`` bf16 activations (T_stage = T * prod(upsample rates so
far)); weights prepacked once as bf16 ``[taps][co_pad][ci_pad]`` for the MFMA implicit-GEMM kernel.
Per stage:  ConvTranspose1d (u polyphase convs, or ONE implicit GEMM with the phases as output
            columns; + conds[i](spk) as a per-utterance bias)
            -> 3 AMPBlock1, each 3 x [act -> conv(dil) -> act -> conv + residual]; the third conv of
               each block also accumulates the block sum and applies the 1/3 mean in its epilogue.
Tail: activation_post -> conv_post + tanh (+ int16 conversion of ``infer()``) in one kernel.

The speaker embedding (ECAPA) and the per-utterance condition biases are per-prompt work done with
PyTorch ops on the device and cached by the caller (quirk Q6).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

from .. import _hip
from .ecapa import speaker_embedding


def fold_weight_norm(sd) -> Dict[str, torch.Tensor]:
    """``remove_weight_norm``: w = g * v / ||v|| with the norm over every dim but 0 (f32)."""
    out = {}
    for k, v in sd.items():
        t = torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
        if k.endswith(".weight_g"):
            continue
        if k.endswith(".weight_v"):
            base = k[: -len(".weight_v")]
            g = torch.as_tensor(np.asarray(sd[base + ".weight_g"])).float() if not isinstance(sd[base + ".weight_g"], torch.Tensor) \
                else sd[base + ".weight_g"].float()
            vv = t.float()
            n = vv.reshape(vv.shape[0], -1).norm(dim=1).reshape(g.shape)
            out[base + ".weight"] = g * vv / n
        else:
            out[k] = t.float() if t.is_floating_point() else t
    return out


def pack_dims(cin: int, cout: int):
    """itts_igemm_pack_dims through the C ABI."""
    lib = _hip.load()
    ci, co = np.zeros(1, np.int32), np.zeros(1, np.int32)
    ci_p = ci.ctypes.data_as(_hip._i32p)
    co_p = co.ctypes.data_as(_hip._i32p)
    _hip.check(lib.itts_igemm_pack_dims(cin, cout, ci_p, co_p), "itts_igemm_pack_dims")
    return int(ci[0]), int(co[0])


def pack_dims_py(cin: int, cout: int):
    """Same contract as itts_igemm_pack_dims (used where the library is not loaded, e.g. CPU tests)."""
    kc = 64 if cin >= 128 else 32
    tn = 128 if cout >= 128 else 32
    return (cin + kc - 1) // kc * kc, (cout + tn - 1) // tn * tn


def pack_taps(taps: List[torch.Tensor], cin: int, cout: int) -> torch.Tensor:
    """taps: list of [cout, cin] f32 matrices -> bf16 [ntaps, co_pad, ci_pad] (zero padded)."""
    ci_pad, co_pad = pack_dims_py(cin, cout)
    out = torch.zeros(len(taps), co_pad, ci_pad, dtype=torch.float32)
    for j, w in enumerate(taps):
        out[j, :cout, :cin] = w
    return out.to(torch.bfloat16)


def conv1d_taps(w: torch.Tensor, dilation: int = 1, padding: int = None):
    """Conv1d weight [co, ci, k] -> (tap matrices, time offsets): y[t] = sum_j W_j x[t + off_j]."""
    k = w.shape[-1]
    pad = dilation * (k - 1) // 2 if padding is None else padding
    return [w[:, :, j] for j in range(k)], [j * dilation - pad for j in range(k)]


def convtr_phases(w: torch.Tensor, u: int, padding: int):
    """ConvTranspose1d weight [ci, co, K], stride u -> per output phase rho (s = u*q + rho):
    (tap matrices [co, ci], input offsets) with y[u*q + rho] = sum_m W_m x[q + off_m]."""
    K = w.shape[-1]
    assert K % u == 0, "kernel must be a multiple of the stride"
    phases = []
    for rho in range(u):
        r = (rho + padding) % u
        base = (rho + padding) // u
        taps = [w[:, :, r + u * m].t().contiguous() for m in range(K // u)]
        offs = [base - m for m in range(K // u)]
        phases.append((taps, offs))
    return phases


def convtr_fused(w: torch.Tensor, u: int, padding: int):
    """ConvTranspose1d as ONE implicit GEMM whose output columns are the u phases: the [T*u][co]
    output viewed as [T][u*co] (row q = output samples u*q .. u*q+u-1, column block rho = phase rho).
    Taps: the union of the phases' input offsets; a phase's block of a tap matrix [u*co, ci] is zero at
    offsets the phase does not use.  The input is read once instead of once per phase."""
    ph = convtr_phases(w, u, padding)
    co, ci = ph[0][0][0].shape
    offs = sorted({o for _, oo in ph for o in oo})
    taps = []
    for o in offs:
        m = torch.zeros(u * co, ci, dtype=torch.float32)
        for rho, (tt, oo) in enumerate(ph):
            if o in oo:
                m[rho * co:(rho + 1) * co] = tt[oo.index(o)]
        taps.append(m)
    return taps, offs


class _Conv:
    def __init__(self, taps, offs, bias, cin, cout, device):
        self.w = pack_taps(taps, cin, cout).to(device)
        self.offs = _hip.i32_array(offs)
        self.ntaps = len(offs)
        self.bias = bias.float().to(device) if bias is not None else None
        self.cin, self.cout = cin, cout


class _Act:
    def __init__(self, sd, prefix, device):
        self.up = sd[prefix + ".upsample.filter"].reshape(-1).float().to(device)
        self.down = sd[prefix + ".downsample.lowpass.filter"].reshape(-1).float().to(device)
        self.alpha = sd[prefix + ".act.alpha"].float().to(device)
        self.beta = sd[prefix + ".act.beta"].float().to(device)
        assert self.up.numel() == 12 and self.down.numel() == 12, "kernel implements the 12-tap Activation1d"


class HipBigVGAN:
    # AMP stage kernels by channel count (measured per conv on MI355X, B=32 x 400 frames,
    # profiles/amp_ab_r02.txt): 24, 48, 96: the MFMA activation kernel + itts_amp_conv_fwd without
    # act (vocoder 101 ms; act fused into the conv for 24 / 48: 107 ms);  others: act + igemm
    FUSED_CHANNELS = ()
    SPLIT_CHANNELS = (24, 48, 96)
    # (round 5 also built conv1 -> act2 of a layer as one launch: bit-identical, measured not faster --
    # profiles/ubench_epi_r05.txt -- and removed in round 6)
    if os.environ.get("ITTS_VOC_FUSED") is not None:  # tuning sweeps: "24,48,96"
        FUSED_CHANNELS = tuple(int(v) for v in os.environ["ITTS_VOC_FUSED"].split(",") if v)
        SPLIT_CHANNELS = tuple(sorted({24, 48, 96} - set(FUSED_CHANNELS)))
    if os.environ.get("ITTS_VOC_SPLIT") is not None:  # channel counts not listed in either: igemm
        SPLIT_CHANNELS = tuple(int(v) for v in os.environ["ITTS_VOC_SPLIT"].split(",") if v)

    def __init__(self, state_dict, cfg_bv, device="cuda"):
        self.lib = _hip.load()
        self.h = h = cfg_bv
        self.device = torch.device(device)
        sd = fold_weight_norm(state_dict)
        self.sd_torch = {k: v.to(self.device) for k, v in sd.items() if k.startswith(("speaker_encoder", "cond_layer", "conds"))}
        dev = self.device
        w = sd["conv_pre.weight"]
        taps, offs = conv1d_taps(w)
        self.conv_pre = _Conv(taps, offs, sd["conv_pre.bias"], w.shape[1], w.shape[0], dev)
        self.ups = []  # (u, convs, C): u phase convs, or ONE conv with the phases as output columns
        for i, (u, k) in enumerate(zip(h.upsample_rates, h.upsample_kernel_sizes)):
            wt = sd[f"ups.{i}.0.weight"]
            u, k = int(u), int(k)
            ci, co = wt.shape[0], wt.shape[1]
            bias = sd[f"ups.{i}.0.bias"]
            if self._fuse_convtr(u, k, co):
                taps, offs = convtr_fused(wt, u, (k - u) // 2)
                convs = [_Conv(taps, offs, bias.reshape(-1).repeat(u), ci, u * co, dev)]
            else:
                convs = [_Conv(t, o, bias, ci, co, dev) for t, o in convtr_phases(wt, u, (k - u) // 2)]
            self.ups.append((u, convs, co))
        self.nk = len(h.resblock_kernel_sizes)
        self.blocks = []
        for i in range(len(h.upsample_rates)):
            stage = []
            for j, (k, dils) in enumerate(zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes)):
                p = f"resblocks.{i * self.nk + j}"
                layers = []
                for n, d in enumerate(dils):
                    w1 = sd[f"{p}.convs1.{n}.weight"]
                    w2 = sd[f"{p}.convs2.{n}.weight"]
                    c1 = _Conv(*conv1d_taps(w1, int(d)), sd[f"{p}.convs1.{n}.bias"], w1.shape[1], w1.shape[0], dev)
                    c2 = _Conv(*conv1d_taps(w2, 1), sd[f"{p}.convs2.{n}.bias"], w2.shape[1], w2.shape[0], dev)
                    layers.append((_Act(sd, f"{p}.activations.{2 * n}", dev), c1,
                                   _Act(sd, f"{p}.activations.{2 * n + 1}", dev), c2))
                stage.append(layers)
            self.blocks.append(stage)
        self.act_post = _Act(sd, "activation_post", dev)
        wp = sd["conv_post.weight"]  # [1, C, K]
        self.post_w = wp[0].contiguous().float().to(dev)
        self.post_b = float(sd["conv_post.bias"].reshape(-1)[0])
        self.post_k = wp.shape[-1]
        self.hop = int(np.prod([int(u) for u in h.upsample_rates]))
        self._bufs = {}
        self._cond_w = {}  # cond_layer / conds[i] weights [out][in] f32 (cond_biases)
        self.fused_amp = True  # narrow stages: activation fused into the conv (False: separate kernels)
        # the whole forward as ONE C-ABI call (itts_bigvgan_forward, bigvgan_fwd.hip) launching the same
        # kernels as _forward_py (ITTS_VOC_CFORWARD=0: the Python launch sequence, the test reference)
        self.cforward = os.environ.get("ITTS_VOC_CFORWARD", "1") != "0"
        self._cw = self._c_weights()
        self._ws = None

    @staticmethod
    def _fuse_convtr(u: int, k: int, co: int) -> bool:
        """All phases in one launch where every phase uses the same input offsets (kernel == stride:
        no extra MFMA work; stages 2 and 3: 4 x 252 -> 451 us and 4 x 85 -> 275 us).  The k = 2u stages
        stay per phase: their offset union has 3 taps instead of 2 per phase (+50 % MFMA); measured at
        C <= 96 too (96: 2 x 470 -> 830 us, 48: 2 x 380 -> 882 us, profiles/convt_ab_r03.txt).
        ITTS_VOC_CONVT_FUSED=0: never; =2: also the narrow k = 2u stages (A/B)."""
        mode = os.environ.get("ITTS_VOC_CONVT_FUSED", "1")
        if u <= 1 or mode == "0":
            return False
        return k == u or (mode == "2" and co <= 96)

    # ---------------- the C-ABI description of this generator ----------------
    @staticmethod
    def _c_conv(c: "_Conv") -> "_hip.Conv":
        offs = (ctypes.c_int32 * 16)(*list(c.offs))
        return _hip.Conv(c.w.data_ptr(), _hip.ptr(c.bias), c.cin, c.cout, c.ntaps, offs)

    @staticmethod
    def _c_act(a: "_Act") -> "_hip.Act":
        return _hip.Act(a.up.data_ptr(), a.down.data_ptr(), a.alpha.data_ptr(), a.beta.data_ptr())

    def _amp_mode(self, C: int) -> int:
        if self.fused_amp and C in self.FUSED_CHANNELS:
            return 1
        if self.fused_amp and C in self.SPLIT_CHANNELS:
            return 2
        return 0

    def _c_weights(self):
        """ItTsBigvganWeights over this generator's packed tensors (arrays kept alive on the struct)."""
        for name in ["cond_layer"] + [f"conds.{i}" for i in range(len(self.ups))]:
            if name not in self._cond_w:
                self._cond_w[name] = self.sd_torch[name + ".weight"][:, :, 0].float().contiguous()
        keep = []
        stages = (_hip.BigvganStage * len(self.ups))()
        for i, (u, convs, C) in enumerate(self.ups):
            ph = (_hip.Conv * len(convs))(*[self._c_conv(c) for c in convs])
            rep = convs[0].cout // C  # fused phases: the speaker bias repeated per phase column block
            blocks = self.blocks[i]
            nl = len(blocks[0])
            lay = (_hip.AmpLayer * (len(blocks) * nl))()
            for j, layers in enumerate(blocks):
                for n, (a1, c1, a2, c2) in enumerate(layers):
                    lay[j * nl + n] = _hip.AmpLayer(self._c_act(a1), self._c_conv(c1), self._c_act(a2), self._c_conv(c2))
            cb = self.sd_torch[f"conds.{i}.bias"].float().repeat(rep).contiguous()
            cw = self._cond_w[f"conds.{i}"].repeat(rep, 1).contiguous()
            keep += [ph, lay, cb, cw]
            stages[i] = _hip.BigvganStage(u, ph, cw.data_ptr(), cb.data_ptr(), len(blocks), nl, lay, self._amp_mode(C))
        pb = self.sd_torch["cond_layer.bias"].float()
        keep += [stages, pb]
        w = _hip.BigvganWeights(len(self.ups), self.conv_pre.cin, self._cond_w["cond_layer"].shape[1],
                                self._c_conv(self.conv_pre), self._cond_w["cond_layer"].data_ptr(), pb.data_ptr(),
                                stages, self._c_act(self.act_post), self.post_w.data_ptr(), self.post_b, self.post_k)
        w._keep = keep
        return w

    # ---------------- per-prompt (cached by the caller) ----------------
    @torch.no_grad()
    def speaker(self, mel_ref: torch.Tensor, fast: bool = False) -> torch.Tensor:
        """mel_ref [B, T, n_mels] -> [B, spk_dim] (ECAPA; PyTorch ops on the device, convolutions as
        im2col GEMMs: run-to-run identical without MIOpen's naive deterministic conv).  fast=True: the
        1x1 convolutions on the bf16 MFMA implicit GEMM (utils/hiplinear.py; the reference's fp16 mode
        runs BigVGAN under autocast, infer.py:613-623)."""
        lin = None
        if fast:
            if getattr(self, "_spk_bank", None) is None:
                from ..utils.hiplinear import HipLinearBank
                self._spk_bank = HipLinearBank(self.sd_torch, self.device)
            lin = self._spk_bank
        return speaker_embedding(self.sd_torch, mel_ref.to(self.device).float(), lin=lin)

    @torch.no_grad()
    def cond_biases(self, spk: torch.Tensor):
        """speaker-embedding biases of conv_pre and of each up-sampling stage (the 1x1 convs
        cond_layer / conds[i] of models.py:184,193-197,224-234) on the exact-f32 GEMM: one fmaf chain
        per output in k order, so an utterance's biases -- and its waveform -- do not depend on which
        other utterances share the batch (a BLAS GEMM picks its algorithm by batch size)."""
        s = spk.float().contiguous()
        B, K = s.shape

        def lin(name):
            w = self._cond_w.get(name)
            if w is None:
                w = self._cond_w[name] = self.sd_torch[name + ".weight"][:, :, 0].float().contiguous()
            y = torch.empty(B, w.shape[0], dtype=torch.float32, device=s.device)
            _hip.check(self.lib.itts_gemm_f32(s.data_ptr(), K, w.data_ptr(), K, B, w.shape[0], K,
                                              self.sd_torch[name + ".bias"].float().data_ptr(), 0, None,
                                              y.data_ptr(), w.shape[0], _hip.stream_ptr()), "itts_gemm_f32")
            return y
        return lin("cond_layer"), [lin(f"conds.{i}") for i in range(len(self.ups))]

    # ---------------- launches ----------------
    def _buf(self, name, shape, dtype=torch.bfloat16):
        key = (name, dtype)
        b = self._bufs.get(key)
        n = int(np.prod(shape))
        if b is None or b.numel() < n:
            b = torch.empty(n, dtype=dtype, device=self.device)
            self._bufs[key] = b
        return b[:n].view(*shape)

    def _act(self, a: _Act, x, y, lens):
        B, T, C = x.shape
        _hip.check(self.lib.itts_aa_snakebeta_fwd(
            x.data_ptr(), y.data_ptr(), a.up.data_ptr(), a.down.data_ptr(), a.alpha.data_ptr(), a.beta.data_ptr(),
            lens.data_ptr(), B, C, T, T * C, C, 1, T * C, C, 1, _hip.dtype_code(x), _hip.dtype_code(y),
            _hip.stream_ptr()), "itts_aa_snakebeta_fwd")

    def _amp(self, c: _Conv, x, y, lens, a: _Act = None, r1=None, r2=None, alpha=1.0):
        """y = alpha * (conv(act(x)) + bias + r1 + r2) in one launch (itts_amp_conv_fwd)."""
        B, T, Cin = x.shape
        Ty = y.shape[1]
        _hip.check(self.lib.itts_amp_conv_fwd(
            x.data_ptr(), T * Cin, Cin, None if a is None else a.up.data_ptr(),
            None if a is None else a.down.data_ptr(), None if a is None else a.alpha.data_ptr(),
            None if a is None else a.beta.data_ptr(), c.w.data_ptr(), c.bias.data_ptr(), _hip.ptr(r1), _hip.ptr(r2),
            y.data_ptr(), Ty * y.shape[2], y.shape[2], lens.data_ptr(), B, T, Cin, c.cout, c.ntaps, c.offs,
            float(alpha), _hip.stream_ptr()), "itts_amp_conv_fwd")

    def _conv(self, c: _Conv, x, y, lens, r1=None, r2=None, alpha=1.0, bias_b=None, ymul=1, yoff=0, Tq=None):
        B, T, Cin = x.shape
        Ty = y.shape[1]
        _hip.check(self.lib.itts_igemm_fwd(
            x.data_ptr(), T * Cin, Cin, c.w.data_ptr(), _hip.ptr(c.bias), _hip.ptr(bias_b), _hip.ptr(r1),
            _hip.ptr(r2), y.data_ptr(), Ty * y.shape[2], y.shape[2], lens.data_ptr(), B, T if Tq is None else Tq,
            Cin, c.cout, c.ntaps, c.offs, ymul, yoff, float(alpha), 0, _hip.dtype_code(y), _hip.stream_ptr()),
            "itts_igemm_fwd")

    @torch.no_grad()
    def forward(self, latent: torch.Tensor, lengths: torch.Tensor, spk: torch.Tensor, want_pcm: bool = True):
        """latent [B, T, gpt_dim] (bf16/f32, device), lengths [B] frames, spk [B, spk_dim]
        -> (wav f32 [B, T*hop], pcm int16 [B, T*hop] or None); samples past lengths*hop are undefined."""
        if not self.cforward:
            return self._forward_py(latent, lengths, spk, want_pcm)
        x = latent.to(self.device)
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        x = x.contiguous()
        B, T, _ = x.shape
        self.rows = int(lengths.sum()) * self.hop  # output rows (host-side, for accounting)
        lens = lengths.to(self.device, torch.int32).contiguous()
        s = spk.to(self.device).float().contiguous()
        nb = int(self.lib.itts_bigvgan_workspace_bytes(ctypes.byref(self._cw), B, T))
        if nb < 0:
            raise _hip.HipError("itts_bigvgan_workspace_bytes: bad sizes")
        if self._ws is None or self._ws.numel() < nb:
            self._ws = None
            self._ws = torch.empty(nb, dtype=torch.uint8, device=self.device)
        wav = torch.empty(B, T * self.hop, dtype=torch.float32, device=self.device)
        pcm = torch.empty(B, T * self.hop, dtype=torch.int16, device=self.device) if want_pcm else None
        _hip.check(self.lib.itts_bigvgan_forward(ctypes.byref(self._cw), x.data_ptr(), lens.data_ptr(), s.data_ptr(),
                                                 B, T, self._ws.data_ptr(), wav.data_ptr(), _hip.ptr(pcm),
                                                 _hip.stream_ptr()), "itts_bigvgan_forward")
        return wav, pcm

    @torch.no_grad()
    def _forward_py(self, latent: torch.Tensor, lengths: torch.Tensor, spk: torch.Tensor, want_pcm: bool = True,
                    taps: dict = None):
        """The same launches from Python (reference for tests/test_gpu_vocoder.py's C-ABI test).
        ``taps`` (tests): filled with copies of the stage boundaries, channel-last bf16 --
        "pre" (conv_pre + cond), "stage{i}" (after upsampling stage i), and the matching lengths."""
        dev = self.device
        x = latent.to(dev)
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        x = x.contiguous()
        B, T, _ = x.shape
        self.rows = int(lengths.sum())  # valid input rows of the current conv (host-side, for FLOP accounting)
        lens = lengths.to(dev, torch.int32).contiguous()
        pre_b, stage_b = self.cond_biases(spk.to(dev))
        C0 = self.conv_pre.cout
        cur_in = self._buf("xs_a", (B, T, C0))
        self._conv(self.conv_pre, x, cur_in, lens, bias_b=pre_b)
        if taps is not None:
            taps["pre"], taps["pre_lens"] = cur_in.clone(), lens.clone()
        Tcur = T
        for i, (u, convs, C) in enumerate(self.ups):
            Tn = Tcur * u
            lens_n = (lens * u).contiguous()
            x_st = self._buf("x", (B, Tn, C))
            if len(convs) == 1 and u > 1:  # phases as output columns: [B][Tcur][u*C] is [B][Tn][C]
                self._conv(convs[0], cur_in, x_st.view(B, Tcur, u * C), lens,
                           bias_b=stage_b[i].repeat(1, u).contiguous())
            else:
                for rho, ph in enumerate(convs):
                    self._conv(ph, cur_in, x_st, lens, bias_b=stage_b[i], ymul=u, yoff=rho)
            self.rows *= u
            t1 = self._buf("t1", (B, Tn, C))
            t2 = self._buf("t2", (B, Tn, C))
            cur = self._buf("cur", (B, Tn, C))
            xs = self._buf("xs_b" if i % 2 == 0 else "xs_a", (B, Tn, C))
            for j, layers in enumerate(self.blocks[i]):
                src = x_st
                fused = self.fused_amp and C in self.FUSED_CHANNELS
                split = self.fused_amp and C in self.SPLIT_CHANNELS
                for n, (a1, c1, a2, c2) in enumerate(layers):
                    last_layer = n == len(layers) - 1
                    alpha = (1.0 / self.nk) if (last_layer and j == self.nk - 1) else 1.0
                    dst = xs if last_layer else cur
                    r2 = xs if (last_layer and j > 0) else None
                    if fused:  # activation fused into each conv's input staging (amp_conv.hip)
                        self._amp(c1, src, t2, lens_n, a1)
                        self._amp(c2, t2, dst, lens_n, a2, r1=src, r2=r2, alpha=alpha)
                    elif split:  # activation kernel + the all-channels conv kernel without activation
                        self._act(a1, src, t1, lens_n)
                        self._amp(c1, t1, t2, lens_n)
                        self._act(a2, t2, t1, lens_n)
                        self._amp(c2, t1, dst, lens_n, r1=src, r2=r2, alpha=alpha)
                    else:
                        self._act(a1, src, t1, lens_n)
                        self._conv(c1, t1, t2, lens_n)
                        self._act(a2, t2, t1, lens_n)
                        self._conv(c2, t1, dst, lens_n, r1=src, r2=r2, alpha=alpha)
                    src = dst
            cur_in, Tcur, lens = xs, Tn, lens_n
            if taps is not None:
                taps[f"stage{i}"], taps[f"stage{i}_lens"] = xs.clone(), lens_n.clone()
        wav = torch.empty(B, Tcur, dtype=torch.float32, device=dev)
        pcm = torch.empty(B, Tcur, dtype=torch.int16, device=dev) if want_pcm else None
        self._tail(cur_in, lens, wav, pcm)
        return wav, pcm

    def tail_fused(self, x) -> bool:
        """activation_post + conv_post + tanh (+ int16) as one launch (itts_act_conv_post_tanh): bf16 channel-last
        input of 8..32 channels (one MFMA channel block; IndexTTS-1.5: 24), the layout the generator runs in"""
        C = x.shape[2]
        return (x.dtype == torch.bfloat16 and C % 8 == 0 and C <= 32 and self.post_k % 2 == 1 and self.post_k <= 15
                and os.environ.get("ITTS_VOC_TAIL_FUSED", "1") != "0")

    def _tail(self, x, lens, wav, pcm, fused=None):
        """wav / pcm = tanh(conv_post(activation_post(x))) (models.py:245-248; int16 as infer.py:627-631):
        one fused launch (bit-identical, tests/test_gpu_vocoder.py), or the activation kernel + itts_conv_post_tanh"""
        B, T, C = x.shape
        if fused if fused is not None else self.tail_fused(x):
            a = self.act_post
            _hip.check(self.lib.itts_act_conv_post_tanh(
                x.data_ptr(), T * C, C, a.up.data_ptr(), a.down.data_ptr(), a.alpha.data_ptr(), a.beta.data_ptr(),
                self.post_w.data_ptr(), self.post_b, C, self.post_k, lens.data_ptr(), B, T, wav.data_ptr(),
                _hip.ptr(pcm), wav.shape[1], _hip.stream_ptr()), "itts_act_conv_post_tanh")
            return
        t1 = self._buf("t1", x.shape)
        self._act(self.act_post, x, t1, lens)
        _hip.check(self.lib.itts_conv_post_tanh(
            t1.data_ptr(), T * C, C, self.post_w.data_ptr(), self.post_b, C, self.post_k, lens.data_ptr(), B, T,
            wav.data_ptr(), _hip.ptr(pcm), wav.shape[1], _hip.dtype_code(t1), _hip.stream_ptr()), "itts_conv_post_tanh")
