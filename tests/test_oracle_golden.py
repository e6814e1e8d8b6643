"""Pin the CPU oracle (and the PyTorch conditioning/ECAPA code) against fixtures produced by the
REFERENCE implementation (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from indextts.gpt.conditioning import get_conditioning
from indextts.utils.config import load_config, default_config_path, tiny_config
from indextts.utils.synthetic import gpt_state_dict, bigvgan_state_dict
from indextts.vocoder.ecapa import speaker_embedding
from oracle.bigvgan_oracle import BigVGANOracle, activation1d, fold_weight_norm, to_int16
from oracle.gpt_oracle import GPTOracle

HEAD_STD = {"tiny": 0.15, "full": 0.08}


def _cfg(tag):
    return tiny_config() if tag == "tiny" else load_config(default_config_path())


_cache = {}


def _gpt(tag):
    if ("gpt", tag) not in _cache:
        cfg = _cfg(tag)
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in gpt_state_dict(cfg.gpt, 0, HEAD_STD[tag]).items()}
        _cache[("gpt", tag)] = (cfg, sd, GPTOracle(sd, cfg.gpt))
    return _cache[("gpt", tag)]


def _bv(tag):
    if ("bv", tag) not in _cache:
        cfg = _cfg(tag)
        sd = bigvgan_state_dict(cfg.bigvgan, 0)
        _cache[("bv", tag)] = (cfg, sd, BigVGANOracle(sd, cfg.bigvgan))
    return _cache[("bv", tag)]


@pytest.mark.parametrize("i", range(5))
def test_activation1d_torch_path(golden, i):
    x = torch.from_numpy(golden[f"act{i}_x"])
    f = torch.from_numpy(golden[f"act{i}_filter"])
    y = activation1d(x, f, f, torch.from_numpy(golden[f"act{i}_alpha"]), torch.from_numpy(golden[f"act{i}_beta"]))
    np.testing.assert_allclose(y.numpy(), golden[f"act{i}_y"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("i", range(6))
def test_remove_long_silence(golden, i):
    codes, lens = GPTOracle.remove_long_silence(torch.from_numpy(golden[f"sil_in_{i}"]))
    np.testing.assert_array_equal(codes.numpy(), golden[f"sil_out_{i}"])
    np.testing.assert_array_equal(lens.numpy(), golden[f"sil_len_{i}"])


@pytest.mark.parametrize("tag", ["tiny", "full"])
def test_conditioning_matches_reference(golden, tag):
    cfg, sd, _ = _gpt(tag)
    mel = torch.from_numpy(golden[f"{tag}_gpt_mel"])
    with torch.no_grad():
        conds = get_conditioning(sd, cfg.gpt, mel)
    np.testing.assert_allclose(conds.numpy(), golden[f"{tag}_gpt_conds"], rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("tag", ["tiny", "full"])
def test_greedy_ids_bit_exact(golden, tag):
    _, _, orc = _gpt(tag)
    conds = torch.from_numpy(golden[f"{tag}_gpt_conds"])
    text = torch.from_numpy(golden[f"{tag}_gpt_text"])
    n = golden[f"{tag}_gpt_codes"].shape[1]
    with torch.no_grad():
        codes = orc.generate(conds, text, n)
        forced = orc.generate(conds, text, n, min_new_tokens=n)
        batch = orc.generate(conds, torch.from_numpy(golden[f"{tag}_gpt_batch_text"]), n)
    np.testing.assert_array_equal(codes.numpy(), golden[f"{tag}_gpt_codes"])
    np.testing.assert_array_equal(forced.numpy(), golden[f"{tag}_gpt_codes_forced"])
    np.testing.assert_array_equal(batch.numpy(), golden[f"{tag}_gpt_codes_batch"])


@pytest.mark.parametrize("tag", ["tiny", "full"])
def test_latent_pass(golden, tag):
    _, _, orc = _gpt(tag)
    conds = torch.from_numpy(golden[f"{tag}_gpt_conds"])
    text = torch.from_numpy(golden[f"{tag}_gpt_text"])
    fixed, lens = orc.remove_long_silence(torch.from_numpy(golden[f"{tag}_gpt_codes_forced"]))
    np.testing.assert_array_equal(fixed.numpy(), golden[f"{tag}_gpt_fixed_codes"])
    with torch.no_grad():
        lat = orc.latent(conds, text, fixed)
    np.testing.assert_allclose(lat.numpy(), golden[f"{tag}_gpt_latent"], rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("tag", ["tiny", "full"])
def test_ecapa_matches_reference(golden, tag):
    cfg, sd, _ = _bv(tag)
    w = {k: torch.from_numpy(np.asarray(v)) for k, v in fold_weight_norm(sd).items()}
    with torch.no_grad():
        spk = speaker_embedding(w, torch.from_numpy(golden[f"{tag}_bv_mel_ref"]))
    np.testing.assert_allclose(spk.numpy(), golden[f"{tag}_bv_spk"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("tag", ["tiny", "full"])
def test_bigvgan_waveform(golden, tag):
    _, _, orc = _bv(tag)
    with torch.no_grad():
        wav = orc.forward(torch.from_numpy(golden[f"{tag}_bv_latent"]), torch.from_numpy(golden[f"{tag}_bv_spk"]))
    ref = golden[f"{tag}_bv_wav"]
    np.testing.assert_allclose(wav.numpy(), ref, rtol=1e-4, atol=5e-5)
    diff = np.abs(to_int16(wav).numpy().astype(np.int32) - golden[f"{tag}_bv_int16"].astype(np.int32))
    assert diff.max() <= 2
