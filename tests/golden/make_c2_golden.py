"""Full-size (benchmark-shape) golden fixtures from the REFERENCE implementation -> golden_c2.npz.

Run in the build container only (``python tests/golden/make_c2_golden.py``); it imports the
reference with the same harness-only shims as ``make_golden.py``.

Config C2 of BASELINE.json at full IndexTTS-1.5 size (``checkpoints/config.yaml``): one utterance,
L = 48 text ids, a 511-frame prompt mel, and

* ``c2_codes``: 400 greedy codes with EOS suppressed (``min_new_tokens=400``, repetition penalty 10),
  so the KV length reaches 32 + 50 + 1 + 400 = 483 -- the C3 decode shape;
* ``c2_top_ids`` / ``c2_top_vals``: the reference's own per-step top-3 ids and scores AFTER its
  logits processors (repetition penalty + min-new-tokens mask), read from HF ``generate``'s
  ``output_scores`` -- the margins the bf16 teacher-forced test exempts near-ties with;
* ``c2_free``: 100 free-running greedy codes (EOS allowed) and ``c2_batch_*``: the
  ``tests/padding_test.py:69-98`` property at full size -- three left-0 / right-1 padded copies
  decoded as ONE batch for 100 steps;
* ``c2_latent``: the teacher-forced latent of the first 64 codes (``return_latent=True``);
* ``c2_bv_*``: BigVGAN2 (full config) on a 64-frame latent with the 511-frame reference mel:
  waveform (65,536 samples) and the reference's int16 conversion (``infer.py:627-631``).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (installs the shims and imports the reference)

N_CODES, N_FREE, L, T_MEL, VOC_T = 400, 100, 48, 511, 64


def main():
    torch.set_num_threads(8)
    full = mg.cfgmod.load_config(os.path.join(mg.REF, "checkpoints", "config.yaml"))
    out = {}
    torch.manual_seed(4321)
    g = mg.ref_gpt(full, 0, mg.GPT_HEAD_STD["full"])
    rng = np.random.default_rng(2024)
    mel = torch.from_numpy(rng.normal(-4.0, 2.0, (1, 100, T_MEL)).astype(np.float32))
    text = torch.from_numpy(rng.integers(2, int(full.gpt.number_text_tokens), (1, L)).astype(np.int32))
    kw = dict(do_sample=False, num_beams=1, repetition_penalty=10.0, top_p=0.8, top_k=None, temperature=1.0,
              num_return_sequences=1, length_penalty=0.0)
    with torch.no_grad():
        conds = g.get_conditioning(mel, torch.tensor([T_MEL]))
        res = g.inference_speech(mel, text, cond_mel_lengths=torch.tensor([T_MEL]), max_generate_length=N_CODES,
                                 min_new_tokens=N_CODES, output_scores=True, return_dict_in_generate=True, **kw)
        codes = res.sequences
        sc = torch.stack([s[0] for s in res.scores], 0)  # [n, V] processed scores
        top = torch.topk(sc, 3, dim=-1)
        assert torch.equal(top.indices[:, 0], codes[0]), "greedy pick != top-1 of the recorded scores"
        free = g.inference_speech(mel, text, cond_mel_lengths=torch.tensor([T_MEL]), max_generate_length=N_FREE, **kw)
        F = torch.nn.functional
        batch = torch.cat([F.pad(text, (5, 0), value=0), F.pad(text, (0, 5), value=1),
                           F.pad(F.pad(text, (2, 0), value=0), (0, 3), value=1)], 0)
        codes_batch = g.inference_speech(mel, batch, cond_mel_lengths=torch.tensor([T_MEL]),
                                         max_generate_length=N_FREE, min_new_tokens=N_FREE, **kw)
        n_lat = VOC_T
        lat_codes = codes[:, :n_lat]
        latent = g(mel, text, torch.tensor([L]), lat_codes, torch.tensor([n_lat]) * g.mel_length_compression,
                   cond_mel_lengths=torch.tensor([T_MEL]), return_latent=True, clip_inputs=False)
    marg = (top.values[:, 0] - top.values[:, 1]).numpy()
    print("c2 codes", tuple(codes.shape), codes[0, :12].tolist(), "margin<=0.1:", int((marg <= 0.1).sum()),
          "min", float(marg.min()), "median", float(np.median(marg)))
    print("free", tuple(free.shape), "batch equal:",
          [bool(torch.equal(codes_batch[i], codes[0, :N_FREE])) for i in range(3)])
    out.update({"c2_mel": mel.numpy(), "c2_text": text.numpy().astype(np.int64), "c2_conds": conds.numpy(),
                "c2_codes": codes.numpy(), "c2_top_ids": top.indices.numpy().astype(np.int32),
                "c2_top_vals": top.values.numpy().astype(np.float32), "c2_free": free.numpy(),
                "c2_batch_text": batch.numpy().astype(np.int64), "c2_codes_batch": codes_batch.numpy(),
                "c2_latent": latent.numpy().astype(np.float32)})
    # vocoder at full config on a 64-frame latent (waveform 65,536 samples)
    m = mg.ref_bigvgan(full, 0)
    vr = np.random.default_rng(2025)
    vlat = torch.from_numpy(vr.normal(0, 1, (1, VOC_T, int(full.bigvgan.gpt_dim))).astype(np.float32))
    mel_ref = torch.from_numpy(vr.normal(-4.0, 2.0, (1, T_MEL, 100)).astype(np.float32))
    with torch.no_grad():
        spk = m.speaker_encoder(mel_ref, None)
        wav, _ = m(vlat, mel_ref)
    out.update({"c2_bv_latent": vlat.numpy(), "c2_bv_mel_ref": mel_ref.numpy(), "c2_bv_spk": spk.squeeze(1).numpy(),
                "c2_bv_wav": wav.numpy(),
                "c2_bv_int16": torch.clamp(32767 * wav, -32767.0, 32767.0).type(torch.int16).numpy()})
    print("c2 wav", tuple(wav.shape), float(wav.abs().max()), float(wav.std()))
    path = os.path.join(HERE, "golden_c2.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
