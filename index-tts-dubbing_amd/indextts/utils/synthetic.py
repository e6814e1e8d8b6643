"""Seeded synthetic checkpoints in the reference's state-dict format.

No IndexTTS weights ship with the reference (``checkpoints/`` only holds ``config.yaml``), so
parity fixtures and the benchmark use deterministic random weights.  Every tensor is drawn from
its own ``numpy.random.Generator(PCG64(seed, crc32(name)))`` stream, so a tensor's values depend
only on (seed, name, shape) -- not on generation order -- and the same dict can be rebuilt on the
GPU box without shipping weights.

Key names and shapes are those of the reference modules' ``state_dict()``:
  * GPT: ``UnifiedVoice`` (``indextts/gpt/model.py:300-386``) with the HF GPT-2 core
    (``build_hf_gpt_transformer`` ``:253-274``; ``wte``/``wpe`` removed), conformer encoder
    (``indextts/gpt/conformer_encoder.py:439-520``) and perceiver (``indextts/gpt/perceiver.py:224``).
  * Vocoder: ``BigVGAN`` (``indextts/BigVGAN/models.py:130-197``) *before* ``remove_weight_norm``,
    i.e. ``weight_g``/``weight_v`` pairs (the format of ``bigvgan_generator.pth``'s "generator").

``mel_head_std`` controls the spread of the mel logits: with plain GPT-2 init the logits are
nearly flat and greedy decoding sits on near-ties, so parity fixtures use a larger value.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict

import numpy as np


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())]))


class _Builder:
    def __init__(self, seed: int):
        self.seed = seed
        self.sd: Dict[str, np.ndarray] = {}

    def normal(self, name, shape, std, mean=0.0):
        self.sd[name] = (_rng(self.seed, name).standard_normal(shape, dtype=np.float32) * np.float32(std)
                         + np.float32(mean)).astype(np.float32)

    def uniform(self, name, shape, lo, hi):
        self.sd[name] = _rng(self.seed, name).uniform(lo, hi, size=shape).astype(np.float32)

    def const(self, name, arr):
        self.sd[name] = np.asarray(arr)

    def linear(self, prefix, n_out, n_in, bias=True, std=None):
        std = (1.0 / math.sqrt(n_in)) if std is None else std
        self.normal(prefix + ".weight", (n_out, n_in), std)
        if bias:
            self.normal(prefix + ".bias", (n_out,), 0.02)

    def layernorm(self, prefix, n):
        self.normal(prefix + ".weight", (n,), 0.05, mean=1.0)
        self.normal(prefix + ".bias", (n,), 0.05)


def sinusoid_table(max_len: int, d: int) -> np.ndarray:
    """ESPnet absolute table ``pe[pos, 2i] = sin(pos / 10000^(2i/d))``, ``pe[pos, 2i+1] = cos(..)``
    (``indextts/gpt/conformer/embedding.py:47-57``), computed in float32 like torch."""
    pos = np.arange(max_len, dtype=np.float32)[:, None]
    div = np.exp(np.arange(0, d, 2, dtype=np.float32) * np.float32(-(math.log(10000.0) / d)))
    pe = np.zeros((max_len, d), dtype=np.float32)
    pe[:, 0::2] = np.sin(pos * div)
    pe[:, 1::2] = np.cos(pos * div)
    return pe[None]


def gpt_state_dict(cfg_gpt, seed: int = 0, mel_head_std: float = 0.02) -> Dict[str, np.ndarray]:
    g = cfg_gpt
    D, L, H = int(g.model_dim), int(g.layers), int(g.heads)
    cm = g.condition_module
    C, FF, CH, NB = int(cm.output_size), int(cm.linear_units), int(cm.attention_heads), int(cm.num_blocks)
    b = _Builder(seed)
    # --- conformer conditioning encoder (conv2d2 subsampling, rel-pos MHA, conv module, FFN) ---
    ce = "conditioning_encoder"
    b.normal(f"{ce}.embed.conv.0.weight", (C, 1, 3, 3), 1.0 / 3.0)
    b.normal(f"{ce}.embed.conv.0.bias", (C,), 0.02)
    b.linear(f"{ce}.embed.out.0", C, C * ((100 - 1) // 2))
    b.const(f"{ce}.embed.pos_enc.pe", sinusoid_table(5000, C))
    b.layernorm(f"{ce}.after_norm", C)
    dk = C // CH
    for i in range(NB):
        p = f"{ce}.encoders.{i}"
        b.normal(f"{p}.self_attn.pos_bias_u", (CH, dk), 0.1)
        b.normal(f"{p}.self_attn.pos_bias_v", (CH, dk), 0.1)
        for n in ("linear_q", "linear_k", "linear_v", "linear_out"):
            b.linear(f"{p}.self_attn.{n}", C, C)
        b.linear(f"{p}.self_attn.linear_pos", C, C, bias=False)
        b.linear(f"{p}.feed_forward.w_1", FF, C)
        b.linear(f"{p}.feed_forward.w_2", C, FF)
        b.normal(f"{p}.conv_module.pointwise_conv1.weight", (2 * C, C, 1), 1.0 / math.sqrt(C))
        b.normal(f"{p}.conv_module.pointwise_conv1.bias", (2 * C,), 0.02)
        b.normal(f"{p}.conv_module.depthwise_conv.weight", (C, 1, 15), 1.0 / math.sqrt(15))
        b.normal(f"{p}.conv_module.depthwise_conv.bias", (C,), 0.02)
        b.layernorm(f"{p}.conv_module.norm", C)
        b.normal(f"{p}.conv_module.pointwise_conv2.weight", (C, C, 1), 1.0 / math.sqrt(C))
        b.normal(f"{p}.conv_module.pointwise_conv2.bias", (C,), 0.02)
        for n in ("norm_ff", "norm_mha", "norm_conv", "norm_final"):
            b.layernorm(f"{p}.{n}", C)
    # --- perceiver resampler (2 layers, 32 latents, GEGLU ff) ---
    pe_ = "perceiver_encoder"
    inner = 64 * CH
    ffi = int(D * int(cm.perceiver_mult) * 2 / 3)
    b.normal(f"{pe_}.latents", (32, D), 0.02 * 25)
    b.linear(f"{pe_}.proj_context", D, C)
    for i in range(2):
        b.linear(f"{pe_}.layers.{i}.0.to_q", inner, D, bias=False)
        b.linear(f"{pe_}.layers.{i}.0.to_kv", 2 * inner, D, bias=False)
        b.linear(f"{pe_}.layers.{i}.0.to_out", D, inner, bias=False)
        b.linear(f"{pe_}.layers.{i}.1.0", 2 * ffi, D)
        b.linear(f"{pe_}.layers.{i}.1.2", D, ffi)
    b.normal(f"{pe_}.norm.gamma", (D,), 0.05, mean=1.0)
    # --- embeddings + GPT-2 core ---
    n_text = int(g.number_text_tokens) + 1
    n_mel = int(g.number_mel_codes)
    b.normal("text_embedding.weight", (n_text, D), 0.5)
    b.normal("mel_embedding.weight", (n_mel, D), 0.5)
    for i in range(L):
        p = f"gpt.h.{i}"
        b.layernorm(f"{p}.ln_1", D)
        # HF Conv1D stores W as [in, out]
        b.normal(f"{p}.attn.c_attn.weight", (D, 3 * D), 1.0 / math.sqrt(D))
        b.normal(f"{p}.attn.c_attn.bias", (3 * D,), 0.02)
        b.normal(f"{p}.attn.c_proj.weight", (D, D), 0.5 / math.sqrt(D * L))
        b.normal(f"{p}.attn.c_proj.bias", (D,), 0.02)
        b.layernorm(f"{p}.ln_2", D)
        b.normal(f"{p}.mlp.c_fc.weight", (D, 4 * D), 1.0 / math.sqrt(D))
        b.normal(f"{p}.mlp.c_fc.bias", (4 * D,), 0.02)
        b.normal(f"{p}.mlp.c_proj.weight", (4 * D, D), 0.5 / math.sqrt(4 * D * L))
        b.normal(f"{p}.mlp.c_proj.bias", (D,), 0.02)
    b.layernorm("gpt.ln_f", D)
    n_mel_pos = int(g.max_mel_tokens) + 2 + 1
    n_text_pos = int(g.max_text_tokens) + 2
    b.normal("mel_pos_embedding.emb.weight", (n_mel_pos, D), 0.5)
    b.normal("text_pos_embedding.emb.weight", (n_text_pos, D), 0.5)
    b.layernorm("final_norm", D)
    b.linear("text_head", n_text, D, std=0.02)
    b.linear("mel_head", n_mel, D, std=mel_head_std)
    return b.sd


def _wn_conv(b: _Builder, prefix: str, shape, std, bias_n):
    """weight-norm parameterised conv: w = g * v / ||v||, norm over all dims but 0."""
    b.normal(prefix + ".weight_v", shape, std)
    v = b.sd[prefix + ".weight_v"]
    nrm = np.sqrt((v.astype(np.float64) ** 2).reshape(shape[0], -1).sum(1))
    jitter = 1.0 + 0.1 * _rng(b.seed, prefix + ".g").standard_normal(shape[0])
    b.sd[prefix + ".weight_g"] = (nrm * jitter).astype(np.float32).reshape(shape[0], *([1] * (len(shape) - 1)))
    b.normal(prefix + ".bias", (bias_n,), 0.02)


def kaiser_sinc_lowpass(cutoff: float, half_width: float, kernel_size: int) -> np.ndarray:
    """Kaiser-windowed sinc low-pass (``alias_free_torch/filter.py:29-58``): even length, centred at
    ``arange(-K/2, K/2) + 0.5``, normalised to unit DC gain. Returned as float32 [1, 1, K]."""
    half = kernel_size // 2
    delta_f = 4 * half_width
    A = 2.285 * (half - 1) * math.pi * delta_f + 7.95
    if A > 50.0:
        beta = 0.1102 * (A - 8.7)
    elif A >= 21.0:
        beta = 0.5842 * (A - 21) ** 0.4 + 0.07886 * (A - 21.0)
    else:
        beta = 0.0
    n = np.arange(kernel_size, dtype=np.float64)
    window = np.i0(beta * np.sqrt(1 - ((2 * n) / (kernel_size - 1) - 1) ** 2)) / np.i0(beta)
    t = np.arange(-half, half, dtype=np.float64) + 0.5
    f = 2 * cutoff * window * np.sinc(2 * cutoff * t)
    f /= f.sum()
    return f.astype(np.float32).reshape(1, 1, kernel_size)


def _ecapa(b: _Builder, prefix: str, n_mels: int, lin: int):
    def tdnn(p, cin, cout, k):
        b.normal(f"{p}.conv.conv.weight", (cout, cin, k), 1.0 / math.sqrt(cin * k))
        b.normal(f"{p}.conv.conv.bias", (cout,), 0.02)
        bn(f"{p}.norm.norm", cout)

    def bn(p, n):
        b.normal(f"{p}.weight", (n,), 0.1, mean=1.0)
        b.normal(f"{p}.bias", (n,), 0.1)
        b.normal(f"{p}.running_mean", (n,), 0.1)
        b.uniform(f"{p}.running_var", (n,), 0.5, 1.5)
        b.const(f"{p}.num_batches_tracked", np.array(0, dtype=np.int64))

    def conv(p, cin, cout):
        b.normal(f"{p}.conv.weight", (cout, cin, 1), 1.0 / math.sqrt(cin))
        b.normal(f"{p}.conv.bias", (cout,), 0.02)

    tdnn(f"{prefix}.blocks.0", n_mels, 512, 5)
    for i, dil in ((1, 2), (2, 3), (3, 4)):
        p = f"{prefix}.blocks.{i}"
        tdnn(f"{p}.tdnn1", 512, 512, 1)
        for j in range(7):
            tdnn(f"{p}.res2net_block.blocks.{j}", 64, 64, 3)
        tdnn(f"{p}.tdnn2", 512, 512, 1)
        conv(f"{p}.se_block.conv1", 512, 128)
        conv(f"{p}.se_block.conv2", 128, 512)
    tdnn(f"{prefix}.mfa", 1536, 1536, 1)
    tdnn(f"{prefix}.asp.tdnn", 1536 * 3, 128, 1)
    conv(f"{prefix}.asp.conv", 128, 1536)
    bn(f"{prefix}.asp_bn.norm", 3072)
    conv(f"{prefix}.fc", 3072, lin)


def bigvgan_state_dict(cfg_bv, seed: int = 0) -> Dict[str, np.ndarray]:
    h = cfg_bv
    b = _Builder(seed + 1000)
    C0 = int(h.upsample_initial_channel)
    spk = int(h.speaker_embedding_dim)
    _wn_conv(b, "conv_pre", (C0, int(h.gpt_dim), 7), 1.0 / math.sqrt(int(h.gpt_dim) * 7), C0)
    for i, (u, k) in enumerate(zip(h.upsample_rates, h.upsample_kernel_sizes)):
        cin, cout = C0 // (2 ** i), C0 // (2 ** (i + 1))
        # ConvTranspose1d weight is [C_in, C_out, k]; each output sees C_in * k / u taps
        _wn_conv(b, f"ups.{i}.0", (cin, cout, int(k)), 1.0 / math.sqrt(cin * int(k) / int(u)), cout)
    filt = kaiser_sinc_lowpass(0.25, 0.3, 12)
    nk = len(h.resblock_kernel_sizes)
    for i in range(len(h.upsample_rates)):
        ch = C0 // (2 ** (i + 1))
        for j, (k, dils) in enumerate(zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes)):
            p = f"resblocks.{i * nk + j}"
            for n in range(len(dils)):
                _wn_conv(b, f"{p}.convs1.{n}", (ch, ch, int(k)), 0.5 / math.sqrt(ch * int(k)), ch)
                _wn_conv(b, f"{p}.convs2.{n}", (ch, ch, int(k)), 0.5 / math.sqrt(ch * int(k)), ch)
            for a in range(2 * len(dils)):
                b.normal(f"{p}.activations.{a}.act.alpha", (ch,), 0.3)
                b.normal(f"{p}.activations.{a}.act.beta", (ch,), 0.3)
                b.const(f"{p}.activations.{a}.upsample.filter", filt.copy())
                b.const(f"{p}.activations.{a}.downsample.lowpass.filter", filt.copy())
    ch = C0 // (2 ** len(h.upsample_rates))
    b.normal("activation_post.act.alpha", (ch,), 0.3)
    b.normal("activation_post.act.beta", (ch,), 0.3)
    b.const("activation_post.upsample.filter", filt.copy())
    b.const("activation_post.downsample.lowpass.filter", filt.copy())
    _wn_conv(b, "conv_post", (1, ch, 7), 0.03 / math.sqrt(ch * 7), 1)  # keep tanh out of saturation
    _ecapa(b, "speaker_encoder", int(h.num_mels), spk)
    b.normal("cond_layer.weight", (C0, spk, 1), 1.0 / math.sqrt(spk))
    b.normal("cond_layer.bias", (C0,), 0.02)
    for i in range(len(h.upsample_rates)):
        chi = C0 // (2 ** (i + 1))
        b.normal(f"conds.{i}.weight", (chi, spk, 1), 1.0 / math.sqrt(spk))
        b.normal(f"conds.{i}.bias", (chi,), 0.02)
    return b.sd


def _plain(d):
    if isinstance(d, dict):
        return {k: _plain(v) for k, v in d.items()}
    if isinstance(d, list):
        return [_plain(v) for v in d]
    return d


def write_checkpoint_dir(path: str, cfg, bpe_model: str, seed: int = 0, mel_head_std: float = 0.08,
                         version: float = 1.5) -> str:
    """A model directory in the reference's layout (``config.yaml``, ``gpt.pth`` = ``{"model": sd}``,
    ``bigvgan_generator.pth`` = ``{"generator": sd}``, ``bpe.model``; ``checkpoints/config.yaml:111-113``)
    holding seeded synthetic weights of ``cfg``'s architecture, so ``IndexTTS(cfg_path, model_dir)``
    -- and every worker process of an ``ITTS_DEVICES`` pool -- can load it like the real checkpoints.
    -> path of the config file."""
    import os
    import shutil

    import torch
    import yaml
    os.makedirs(path, exist_ok=True)
    cfg = _plain(cfg)
    cfg["version"] = version
    with open(os.path.join(path, "config.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    from .config import AttrDict
    acfg = AttrDict(cfg)
    t = lambda sd: {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}  # noqa: E731
    torch.save({"model": t(gpt_state_dict(acfg.gpt, seed, mel_head_std))}, os.path.join(path, acfg.gpt_checkpoint))
    torch.save({"generator": t(bigvgan_state_dict(acfg.bigvgan, seed))}, os.path.join(path, acfg.bigvgan_checkpoint))
    shutil.copy(bpe_model, os.path.join(path, acfg.dataset["bpe_model"]))
    return os.path.join(path, "config.yaml")
