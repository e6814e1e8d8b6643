"""ORACLE (test infrastructure only -- never imported by the product path).

CPU fp32 restatement of the BigVGAN2 speech-code -> waveform generator as the reference runs it
(torch path of the anti-aliased activation, quirk Q7).  Layout follows the reference: [B, C, T].

Reference anchors (paths relative to the reference tree):
  * weight-norm fold w = g * v / ||v|| (norm over dims != 0)        torch.nn.utils.remove_weight_norm; BigVGAN/models.py:252-260
  * BigVGAN.forward: conv_pre + cond_layer(spk) -> 6 x [ups + conds(spk), mean of 3 AMPBlock1]
    -> activation_post -> conv_post -> tanh                          BigVGAN/models.py:201-250
  * AMPBlock1.forward: x += c2(a2(c1(a1(x)))) for dil 1,3,5          BigVGAN/models.py:65-74
  * zero "same" padding d*(k-1)/2                                     BigVGAN/utils.py:59-60
  * Activation1d = UpSample1d(2,12) -> SnakeBeta -> DownSample1d(2,12) alias_free_torch/act.py:24-29
  * UpSample1d: replicate pad 5 -> 2*conv_transpose1d(stride 2) -> crop 15/15   alias_free_torch/resample.py:25-33
  * DownSample1d: replicate pad 5/6 -> conv1d(stride 2)              alias_free_torch/filter.py:87-96
  * SnakeBeta (log-scale): x + 1/(exp(b)+1e-9) * sin(x*exp(a))^2      BigVGAN/activations.py:109-122
  * output int16: clamp(32767*wav, +-32767) then truncating cast (Q8) infer.py:627-660
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F


def fold_weight_norm(sd: Dict[str, object]) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in sd.items():
        t = torch.as_tensor(v)
        if k.endswith(".weight_g"):
            continue
        if k.endswith(".weight_v"):
            base = k[: -len(".weight_v")]
            g = torch.as_tensor(sd[base + ".weight_g"]).float()
            vv = t.float()
            nrm = vv.reshape(vv.shape[0], -1).norm(dim=1).reshape(g.shape)
            out[base + ".weight"] = g * vv / nrm
        else:
            out[k] = t.float() if t.is_floating_point() else t
    return out


def snake_beta(x, log_alpha, log_beta):
    a = torch.exp(log_alpha)[None, :, None]
    b = torch.exp(log_beta)[None, :, None]
    return x + (1.0 / (b + 1e-9)) * torch.sin(x * a).pow(2)


def activation1d(x, up_filter, down_filter, log_alpha, log_beta):
    C = x.shape[1]
    K = up_filter.shape[-1]
    pad = K // 2 - 1
    y = F.pad(x, (pad, pad), mode="replicate")
    y = 2.0 * F.conv_transpose1d(y, up_filter.reshape(1, 1, K).expand(C, -1, -1), stride=2, groups=C)
    crop_l = pad * 2 + (K - 2) // 2
    crop_r = pad * 2 + (K - 2 + 1) // 2
    y = y[..., crop_l:-crop_r]
    y = snake_beta(y, log_alpha, log_beta)
    y = F.pad(y, (K // 2 - 1, K // 2), mode="replicate")
    return F.conv1d(y, down_filter.reshape(1, 1, K).expand(C, -1, -1), stride=2, groups=C)


class BigVGANOracle:
    def __init__(self, sd, cfg_bv):
        self.sd = fold_weight_norm(sd)
        self.h = cfg_bv

    def act(self, prefix, x):
        sd = self.sd
        return activation1d(x, sd[prefix + ".upsample.filter"], sd[prefix + ".downsample.lowpass.filter"],
                            sd[prefix + ".act.alpha"], sd[prefix + ".act.beta"])

    def conv(self, prefix, x, dilation=1):
        w = self.sd[prefix + ".weight"]
        k = w.shape[-1]
        return F.conv1d(x, w, self.sd[prefix + ".bias"], dilation=dilation, padding=dilation * (k - 1) // 2)

    def amp_block(self, idx, x, k, dils):
        p = f"resblocks.{idx}"
        for n, d in enumerate(dils):
            xt = self.act(f"{p}.activations.{2 * n}", x)
            xt = self.conv(f"{p}.convs1.{n}", xt, d)
            xt = self.act(f"{p}.activations.{2 * n + 1}", xt)
            xt = self.conv(f"{p}.convs2.{n}", xt, 1)
            x = xt + x
        return x

    def pre(self, latent, spk):
        """conv_pre + cond_layer (models.py:220-226): latent [B, T, gpt_dim] -> [B, C0, T]."""
        sd = self.sd
        x = self.conv("conv_pre", latent.float().transpose(1, 2))
        return x + F.conv1d(spk.float()[:, :, None], sd["cond_layer.weight"], sd["cond_layer.bias"])

    def stage(self, i, x, spk):
        """upsampling stage i (models.py:228-243): ups[i] + conds[i], then the mean of the AMP blocks."""
        sd, h = self.sd, self.h
        u, k = int(h.upsample_rates[i]), int(h.upsample_kernel_sizes[i])
        x = F.conv_transpose1d(x, sd[f"ups.{i}.0.weight"], sd[f"ups.{i}.0.bias"], stride=u, padding=(k - u) // 2)
        x = x + F.conv1d(spk.float()[:, :, None], sd[f"conds.{i}.weight"], sd[f"conds.{i}.bias"])
        nk = len(h.resblock_kernel_sizes)
        xs = None
        for j, (kk, dils) in enumerate(zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes)):
            r = self.amp_block(i * nk + j, x, int(kk), [int(d) for d in dils])
            xs = r if xs is None else xs + r
        return xs / nk

    def post(self, x):
        """activation_post -> conv_post -> tanh (models.py:246-248)."""
        return torch.tanh(self.conv("conv_post", self.act("activation_post", x)))

    def forward(self, latent, spk):
        """latent [B, T, gpt_dim], spk [B, spk_dim] -> wav [B, 1, T * prod(upsample_rates)] float32
        (BigVGAN.forward, models.py:201-250: pre, the upsampling stages, post)."""
        x = self.pre(latent, spk)
        for i in range(len(self.h.upsample_rates)):
            x = self.stage(i, x, spk)
        return self.post(x)


def to_int16(wav: torch.Tensor) -> torch.Tensor:
    """``torch.clamp(32767 * wav, -32767, 32767).type(torch.int16)`` (truncation toward zero)."""
    return torch.clamp(32767 * wav, -32767.0, 32767.0).to(torch.int16)
