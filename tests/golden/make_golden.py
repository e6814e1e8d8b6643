"""Generate the golden fixtures in tests/golden/ by running the REFERENCE implementation.

Run in the build container only (the reference tree is mounted at /root/reference there; it never
travels to the GPU box):  ``python tests/golden/make_golden.py``

The reference is imported unmodified with harness-only shims:
  1. a stub ``torchaudio`` module (imported but unused on these paths; torchaudio is absent),
  2. a stub ``transformers.utils.model_parallel_utils`` (removed in transformers 5.x; only used by
     the never-called ``parallelize``),
  3. a prefill shim on ``prepare_inputs_for_generation`` that passes an empty cache as ``None``
     (transformers 4.36 semantics; without it 5.x silently drops the conditioning prefix),
  4. a stub ``omegaconf`` module so ``indextts/infer.py`` imports (only its pure-tensor
     ``remove_long_silence`` method is exercised, on an instance created without ``__init__``).
Weights are the seeded synthetic state dicts of ``indextts.utils.synthetic`` loaded with
``load_state_dict(strict=True)``.  Only inputs and outputs are stored (npz, float32/int64).
"""
from __future__ import annotations

import importlib.machinery
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "index-tts-dubbing_amd"))
REF = os.environ.get("ITTS_REFERENCE", "/root/reference")

import transformers  # noqa: E402  (must precede the torchaudio stub)

_ta = types.ModuleType("torchaudio")
_ta.__spec__ = importlib.machinery.ModuleSpec("torchaudio", None)
sys.modules.setdefault("torchaudio", _ta)
_mpu = types.ModuleType("transformers.utils.model_parallel_utils")
_mpu.assert_device_map = _mpu.get_device_map = lambda *a, **k: None
sys.modules["transformers.utils.model_parallel_utils"] = _mpu
_oc = types.ModuleType("omegaconf")  # imported by indextts/infer.py; only remove_long_silence is used
_oc.OmegaConf = None
sys.modules.setdefault("omegaconf", _oc)
sys.path.insert(0, REF)

from indextts.BigVGAN.models import BigVGAN as RefBigVGAN  # noqa: E402
from indextts.BigVGAN.alias_free_torch import Activation1d as RefAct1d  # noqa: E402
from indextts.BigVGAN.activations import SnakeBeta as RefSnakeBeta  # noqa: E402
from indextts.gpt.model import UnifiedVoice  # noqa: E402
import indextts.infer as ref_infer_mod  # noqa: E402

# the reference package shadows ours under the same name; load our utils by path
import importlib.util  # noqa: E402


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


PKG = os.path.join(REPO, "index-tts-dubbing_amd", "indextts")
cfgmod = _load("itts_cfg", os.path.join(PKG, "utils", "config.py"))
synth = _load("itts_synth", os.path.join(PKG, "utils", "synthetic.py"))

GPT_HEAD_STD = {"tiny": 0.15, "full": 0.08}


def to_t(sd):
    return {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}


def ref_gpt(cfg, seed, head_std):
    g = UnifiedVoice(**cfg.gpt)
    g.load_state_dict(to_t(synth.gpt_state_dict(cfg.gpt, seed=seed, mel_head_std=head_std)), strict=True)
    g.eval()
    g.post_init_gpt2_config(use_deepspeed=False, kv_cache=True, half=False)
    im = g.inference_model
    orig = im.prepare_inputs_for_generation

    def prep(input_ids, past_key_values=None, **kwargs):  # shim 3 (HF inspects the name "kwargs")
        if past_key_values is not None and hasattr(past_key_values, "get_seq_length") \
                and past_key_values.get_seq_length() == 0:
            past_key_values = None
        return orig(input_ids, past_key_values=past_key_values, **kwargs)

    im.prepare_inputs_for_generation = prep
    return g


def ref_bigvgan(cfg, seed):
    m = RefBigVGAN(cfg.bigvgan, use_cuda_kernel=False)
    m.load_state_dict(to_t(synth.bigvgan_state_dict(cfg.bigvgan, seed=seed)), strict=True)
    m.remove_weight_norm()
    return m.eval()


def greedy(g, mel, text, n, min_new=0):
    kw = dict(do_sample=False, num_beams=1, repetition_penalty=10.0, max_generate_length=n, top_p=0.8,
              top_k=None, temperature=1.0, num_return_sequences=1, length_penalty=0.0)
    if min_new:
        kw["min_new_tokens"] = min_new
    return g.inference_speech(mel, text, cond_mel_lengths=torch.tensor([mel.shape[-1]]), **kw)


def gpt_fixture(tag, cfg, seed, n_steps, T_mel, L, out):
    torch.manual_seed(1234 + seed)
    g = ref_gpt(cfg, seed, GPT_HEAD_STD[tag])
    rng = np.random.default_rng(100 + seed)
    mel = torch.from_numpy(rng.normal(-4.0, 2.0, (1, 100, T_mel)).astype(np.float32))
    text = torch.from_numpy(rng.integers(2, int(cfg.gpt.number_text_tokens), (1, L)).astype(np.int32))
    with torch.no_grad():
        conds = g.get_conditioning(mel, torch.tensor([T_mel]))
        codes = greedy(g, mel, text, n_steps)
        codes_forced = greedy(g, mel, text, n_steps, min_new=n_steps)
        # padding_test.py-style batch: left-0 / right-1 padded copies decoded as ONE batch
        padded = [torch.nn.functional.pad(text, (3, 0), value=0), torch.nn.functional.pad(text, (0, 3), value=1),
                  torch.nn.functional.pad(torch.nn.functional.pad(text, (1, 0), value=0), (0, 2), value=1)]
        batch = torch.cat(padded, 0)
        codes_batch = greedy(g, mel, batch, n_steps)
        tts = ref_infer_mod.IndexTTS.__new__(ref_infer_mod.IndexTTS)
        tts.stop_mel_token = int(cfg.gpt.stop_mel_token)
        fixed, lens = tts.remove_long_silence(codes_forced.clone(), silent_token=52, max_consecutive=30)
        latent = g(mel, text, torch.tensor([L]), fixed, lens * g.mel_length_compression,
                   cond_mel_lengths=torch.tensor([T_mel]), return_latent=True, clip_inputs=False)
    out.update({
        f"{tag}_gpt_mel": mel.numpy(), f"{tag}_gpt_text": text.numpy().astype(np.int64),
        f"{tag}_gpt_conds": conds.numpy(), f"{tag}_gpt_codes": codes.numpy(),
        f"{tag}_gpt_codes_forced": codes_forced.numpy(), f"{tag}_gpt_batch_text": batch.numpy().astype(np.int64),
        f"{tag}_gpt_codes_batch": codes_batch.numpy(), f"{tag}_gpt_latent": latent.numpy(),
        f"{tag}_gpt_fixed_codes": fixed.numpy(), f"{tag}_gpt_fixed_lens": lens.numpy(),
    })
    print(tag, "codes", codes.shape, codes[0, :16].tolist(), "batch equal:",
          [bool(torch.equal(codes_batch[i, :codes.shape[1]], codes[0])) for i in range(3)], "latent", tuple(latent.shape))


def silence_fixture(out):
    """remove_long_silence on constructed code rows (token 52 runs, stop tokens, padding)."""
    tts = ref_infer_mod.IndexTTS.__new__(ref_infer_mod.IndexTTS)
    tts.stop_mel_token = 8193
    rng = np.random.default_rng(7)
    cases = []
    for case in range(6):
        n = int(rng.integers(20, 90))
        row = rng.integers(0, 8192, n)
        if case % 2 == 0:  # many silent tokens in runs
            for _ in range(int(rng.integers(3, 7))):
                s = int(rng.integers(0, n - 1))
                row[s: s + int(rng.integers(5, 25))] = 52
        if case in (1, 2, 4):
            cut = int(rng.integers(5, n))
            row[cut:] = 8193
        cases.append(torch.from_numpy(row.astype(np.int64))[None])
    for i, c in enumerate(cases):
        fixed, lens = tts.remove_long_silence(c.clone(), silent_token=52, max_consecutive=30)
        out[f"sil_in_{i}"] = c.numpy()
        out[f"sil_out_{i}"] = fixed.numpy()
        out[f"sil_len_{i}"] = lens.numpy()


def bigvgan_fixture(tag, cfg, seed, T, Tm, out):
    m = ref_bigvgan(cfg, seed)
    rng = np.random.default_rng(200 + seed)
    latent = torch.from_numpy(rng.normal(0, 1, (1, T, int(cfg.bigvgan.gpt_dim))).astype(np.float32))
    mel_ref = torch.from_numpy(rng.normal(-4.0, 2.0, (1, Tm, 100)).astype(np.float32))
    with torch.no_grad():
        spk = m.speaker_encoder(mel_ref, None)
        wav, _ = m(latent, mel_ref)
    out.update({f"{tag}_bv_latent": latent.numpy(), f"{tag}_bv_mel_ref": mel_ref.numpy(),
                f"{tag}_bv_spk": spk.squeeze(1).numpy(), f"{tag}_bv_wav": wav.numpy(),
                f"{tag}_bv_int16": torch.clamp(32767 * wav, -32767.0, 32767.0).type(torch.int16).numpy()})
    print(tag, "wav", tuple(wav.shape), float(wav.abs().max()), float(wav.std()))


def act_fixture(out):
    """Activation1d (torch path) per-op vectors, incl. T=1..3 edge cases."""
    rng = np.random.default_rng(11)
    for i, (B, C, T) in enumerate([(2, 96, 300), (1, 24, 7), (1, 8, 1), (3, 5, 2), (1, 48, 1029)]):
        a = RefAct1d(activation=RefSnakeBeta(C, alpha_logscale=True))
        with torch.no_grad():
            a.act.alpha.copy_(torch.from_numpy(rng.normal(0, 0.5, C).astype(np.float32)))
            a.act.beta.copy_(torch.from_numpy(rng.normal(0, 0.5, C).astype(np.float32)))
            x = torch.from_numpy(rng.normal(0, 1.5, (B, C, T)).astype(np.float32))
            y = a(x)
        out[f"act{i}_x"] = x.numpy()
        out[f"act{i}_alpha"] = a.act.alpha.detach().numpy()
        out[f"act{i}_beta"] = a.act.beta.detach().numpy()
        out[f"act{i}_y"] = y.numpy()
        out[f"act{i}_filter"] = a.upsample.filter.numpy()


def main():
    torch.set_num_threads(8)
    tiny = cfgmod.tiny_config()
    full = cfgmod.load_config(os.path.join(REF, "checkpoints", "config.yaml"))
    out = {}
    act_fixture(out)
    silence_fixture(out)
    gpt_fixture("tiny", tiny, 0, 40, 137, 12, out)
    bigvgan_fixture("tiny", tiny, 0, 9, 61, out)
    gpt_fixture("full", full, 0, 24, 80, 12, out)
    bigvgan_fixture("full", full, 0, 5, 53, out)
    path = os.path.join(HERE, "golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
