"""Golden fixtures for beam-search decoding, produced by running the REFERENCE ``inference_speech``
(gpt/model.py:655-708) with ``num_beams=3, do_sample=False`` through the installed transformers.

Run in the build container only:  ``python tests/golden/make_beam_golden.py``  -> beam_golden.npz

Harness shims: those of make_golden.py, plus the cache reorder of SURVEY.md §8(c) shim 4 (the
reference's legacy tuple ``_reorder_cache`` does not accept transformers 5.x cache objects).
The reference pins transformers 4.36.2, whose beam search was rewritten in 4.5x; for beam search
without sampling at length_penalty=0 (IndexTTS's default) the rewrite selects the same sequences
(top-2K continuations, eos only from the top K, early stop once no open beam can beat the worst
finished one), so these fixtures pin the oracle's 4.36 restatement (oracle/gpt_oracle.py
``generate_beam``).  Beam *sampling* draws cannot be pinned (RNG streams differ); it is tested
statistically.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (installs the shims, imports the reference)


def ref_gpt_beam(cfg, seed, head_std, eos_boost=0.0):
    g = mg.ref_gpt(cfg, seed, head_std)
    with torch.no_grad():  # raise the stop logit so that hypotheses close within the step budget
        g.mel_head.bias[int(cfg.gpt.stop_mel_token)] += eos_boost
    im = g.inference_model

    def reorder(past, beam_idx):  # shim 4
        if hasattr(past, "reorder_cache"):
            past.reorder_cache(beam_idx)
            return past
        return type(im)._reorder_cache(past, beam_idx)

    im._reorder_cache = reorder
    return g


def beam(g, mel, text, n, K=3, min_new=0):
    kw = dict(do_sample=False, num_beams=K, repetition_penalty=10.0, max_generate_length=n, top_p=None,
              top_k=None, temperature=None, num_return_sequences=1, length_penalty=0.0)
    if min_new:
        kw["min_new_tokens"] = min_new
    return g.inference_speech(mel, text, cond_mel_lengths=torch.tensor([mel.shape[-1]]), **kw)


def fixture(tag, cfg, seed, n_steps, T_mel, L, out, head_std):
    torch.manual_seed(1234 + seed)
    g = ref_gpt_beam(cfg, seed, head_std)
    rng = np.random.default_rng(300 + seed)
    mel = torch.from_numpy(rng.normal(-4.0, 2.0, (1, 100, T_mel)).astype(np.float32))
    text = torch.from_numpy(rng.integers(2, int(cfg.gpt.number_text_tokens), (1, L)).astype(np.int32))
    padded = [torch.nn.functional.pad(text, (2, 0), value=0), torch.nn.functional.pad(text, (0, 2), value=1)]
    batch = torch.cat(padded + [torch.from_numpy(rng.integers(2, int(cfg.gpt.number_text_tokens), (1, L + 2))
                                                 .astype(np.int32))], 0)
    with torch.no_grad():
        conds = g.get_conditioning(mel, torch.tensor([T_mel]))
        codes = beam(g, mel, text, n_steps)
        codes_k2 = beam(g, mel, text, n_steps, K=2)
        codes_batch = beam(g, mel, batch, n_steps)
        codes_forced = beam(g, mel, text, n_steps, min_new=n_steps // 2)
    out.update({f"{tag}_mel": mel.numpy(), f"{tag}_text": text.numpy().astype(np.int64),
                f"{tag}_conds": conds.numpy(), f"{tag}_codes": codes.numpy(), f"{tag}_codes_k2": codes_k2.numpy(),
                f"{tag}_batch_text": batch.numpy().astype(np.int64), f"{tag}_codes_batch": codes_batch.numpy(),
                f"{tag}_codes_minnew": codes_forced.numpy(), f"{tag}_steps": np.array(n_steps),
                f"{tag}_head_std": np.array(head_std)})
    print(tag, "codes", tuple(codes.shape), codes[0, :12].tolist(), "k2", tuple(codes_k2.shape), "batch",
          tuple(codes_batch.shape), "minnew", tuple(codes_forced.shape))


def eos_fixture(tag, cfg, seed, n_steps, boost, out, head_std):
    """same inputs as ``fixture`` with the stop logit raised by ``boost`` (bias of mel_head): eos
    candidates close hypotheses mid-run, utterances finish at different steps, early stop fires."""
    g = ref_gpt_beam(cfg, seed, head_std, boost)
    mel = torch.from_numpy(out[f"{tag}_mel"])
    batch = torch.from_numpy(out[f"{tag}_batch_text"]).int()
    with torch.no_grad():
        codes = beam(g, mel, batch, n_steps)
    out[f"{tag}_eos{boost:g}_codes_batch"] = codes.numpy()
    print(tag, "eos boost", boost, tuple(codes.shape), [int((r == 8193).nonzero()[0]) if (r == 8193).any() else None
                                                         for r in codes])


def main():
    torch.set_num_threads(8)
    tiny = mg.cfgmod.tiny_config()
    full = mg.cfgmod.load_config(os.path.join(mg.REF, "checkpoints", "config.yaml"))
    out = {}
    # head std chosen so that eos competes within the step budget (hypotheses close mid-run)
    fixture("tiny", tiny, 0, 40, 137, 12, out, 0.15)
    fixture("full", full, 0, 20, 80, 12, out, 0.08)
    for b in (5.0, 6.0):
        eos_fixture("tiny", tiny, 0, 40, b, out, 0.15)
    for b in (4.0, 6.0):
        eos_fixture("full", full, 0, 20, b, out, 0.08)
    path = os.path.join(HERE, "beam_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
