"""Model config loading.

The reference loads ``checkpoints/config.yaml`` with OmegaConf (``indextts/infer.py:56``) and
relies on attribute access (``cfg.gpt.stop_mel_token``), ``h.get(...)`` and item assignment
(``h["use_cuda_kernel"] = ...`` in ``indextts/BigVGAN/models.py:140``).  OmegaConf is not part
of this image, so this module provides the same surface on top of ``yaml.safe_load``.
"""
from __future__ import annotations

import copy
import os

import yaml


class AttrDict(dict):
    """dict with attribute access, recursively applied (OmegaConf DictConfig look-alike)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        for k, v in list(self.items()):
            self[k] = _wrap(v)

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as e:
            raise AttributeError(key) from e

    def __setattr__(self, key, value):
        self[key] = _wrap(value)

    def __deepcopy__(self, memo):
        return AttrDict({k: copy.deepcopy(v, memo) for k, v in self.items()})


def _wrap(v):
    if isinstance(v, AttrDict):
        return v
    if isinstance(v, dict):
        return AttrDict(v)
    if isinstance(v, list):
        return [_wrap(x) for x in v]
    return v


def load_config(path: str) -> AttrDict:
    with open(path, "r", encoding="utf-8") as f:
        return AttrDict(yaml.safe_load(f))


def default_config_path() -> str:
    """Path of the bundled copy of the reference's ``checkpoints/config.yaml`` (IndexTTS-1.5)."""
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "config.yaml")


def tiny_config() -> AttrDict:
    """A scaled-down config with the same structure, used by parity fixtures.

    Head size (64), the mel-code vocabulary (8194, stop 8193, start 8192, silent 52) and the
    anti-alias filters are kept so every code path and special token of the real model is hit.
    """
    cfg = load_config(default_config_path())
    g = cfg.gpt
    g.model_dim = 256
    g.heads = 4
    g.layers = 2
    g.condition_module.output_size = 128
    g.condition_module.linear_units = 256
    g.condition_module.attention_heads = 2
    g.condition_module.num_blocks = 2
    b = cfg.bigvgan
    b.upsample_initial_channel = 192
    b.gpt_dim = 256
    return cfg
