"""GPU tests of the drop-in ``IndexTTS`` (indextts/infer.py) and of the sampling kernel.

* ``IndexTTS.infer`` / ``infer_fast`` on a synthetic tiny checkpoint directory, f32 mode, greedy:
  output length must equal the oracle chain's (prompt mel -> conditioning -> GPTOracle greedy ids
  per sentence -> remove_long_silence -> latent -> BigVGANOracle -> int16) exactly (bit-exact ids);
  the int16 waveform within the vocoder tolerance of tests/test_gpu_vocoder.py (bf16 vocoder
  storage: relative RMS <= 2e-2).
* ``itts_sample_topk_embed``: empirical token frequencies over >= 40k draws vs. the probabilities
  of HF's Temperature -> TopK -> TopP warpers computed in torch fp32 (|f - p| <= 5 sigma + 2e-3,
  zero draws outside the kept set); ties at the k-th value are kept; a fixed seed reproduces the
  draws (graph replay == eager).
"""
import os
import shutil
import wave

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _plain(d):
    if isinstance(d, dict):
        return {k: _plain(v) for k, v in d.items()}
    if isinstance(d, list):
        return [_plain(v) for v in d]
    return d


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    import yaml
    from indextts.utils.config import tiny_config
    from indextts.utils.synthetic import bigvgan_state_dict, gpt_state_dict
    d = tmp_path_factory.mktemp("ckpt")
    cfg = tiny_config()
    cfg.version = 1.5
    with open(d / "config.yaml", "w") as f:
        yaml.safe_dump(_plain(cfg), f)
    t = lambda sd: {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}  # noqa: E731
    gsd, bsd = t(gpt_state_dict(cfg.gpt, 0, 0.15)), t(bigvgan_state_dict(cfg.bigvgan, 0))
    torch.save({"model": gsd}, d / "gpt.pth")
    torch.save({"generator": bsd}, d / "bigvgan_generator.pth")
    shutil.copy(os.path.join(HERE, "golden", "tiny_bpe.model"), d / "bpe.model")
    # prompt: 1.5 s of a chirp + noise at 16 kHz, stereo (exercises mono mix + resampling)
    sr, n = 16000, 24000
    tt = np.arange(n) / sr
    rng = np.random.default_rng(0)
    sig = 0.3 * np.sin(2 * np.pi * (150 + 200 * tt) * tt) + 0.05 * rng.standard_normal(n)
    pcm = (np.stack([sig, 0.8 * sig], 1) * 32767).astype("<i2")
    with wave.open(str(d / "prompt.wav"), "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm.tobytes())
    return d, cfg, gsd, bsd


def _oracle_chain(ckpt, text, max_mel_tokens, max_tokens, fast):
    from indextts.gpt.conditioning import get_conditioning
    from indextts.utils.audio import prompt_mel
    from indextts.utils.text import TextNormalizer, TextTokenizer
    from indextts.vocoder.ecapa import speaker_embedding
    from oracle.bigvgan_oracle import BigVGANOracle, fold_weight_norm, to_int16
    from oracle.gpt_oracle import GPTOracle
    d, cfg, gsd, bsd = ckpt
    norm = TextNormalizer()
    norm.load()
    tok = TextTokenizer(str(d / "bpe.model"), norm)
    sents = tok.split_sentences(tok.tokenize(text), max_tokens)
    mel = prompt_mel(str(d / "prompt.wav"))
    g = GPTOracle(gsd, cfg.gpt)
    bv = BigVGANOracle(bsd, cfg.bigvgan)
    with torch.no_grad():
        conds = get_conditioning({k: v.float() for k, v in gsd.items()}, cfg.gpt, mel)
        spk = speaker_embedding(fold_weight_norm(bsd), mel.transpose(1, 2))
        lat = []
        for s in sents:
            ids = torch.tensor([tok.convert_tokens_to_ids(s)])
            codes = g.generate(conds, ids, max_mel_tokens)
            codes, _ = GPTOracle.remove_long_silence(codes)
            lat.append(g.latent(conds, ids, codes))
        if fast:
            lat = [torch.cat(lat[i: i + 2], 1) for i in range(0, len(lat), 2)]
        wavs = [to_int16(bv.forward(x, spk))[0, 0] for x in lat]
    return torch.cat(wavs).numpy(), len(sents)


def _read_wav(path):
    with wave.open(str(path), "rb") as w:
        assert (w.getnchannels(), w.getsampwidth(), w.getframerate()) == (1, 2, 24000)
        return np.frombuffer(w.readframes(w.getnframes()), dtype="<i2")


def _close(got, want):
    assert got.shape == want.shape
    g, w = got.astype(np.float64), want.astype(np.float64)
    rel = np.sqrt(np.mean((g - w) ** 2)) / max(np.sqrt(np.mean(w ** 2)), 1.0)
    assert rel <= 2e-2, rel


TEXT = "There is a vehicle arriving in dock number 7? Please stand clear. The doors are closing - mind the gap!"


@pytest.fixture(scope="module")
def tts(ckpt):
    from indextts.infer import IndexTTS
    d = ckpt[0]
    return IndexTTS(cfg_path=str(d / "config.yaml"), model_dir=str(d), is_fp16=False, device="cuda:0")


@pytest.mark.parametrize("fast", [False, True])
def test_infer_matches_oracle_chain(ckpt, tts, tmp_path, fast):
    gen = dict(do_sample=False, num_beams=1, max_mel_tokens=40)
    want, nsent = _oracle_chain(ckpt, TEXT, 40, 12, fast)
    assert nsent >= 3
    fn = tts.infer_fast if fast else tts.infer
    sr, got = fn(str(ckpt[0] / "prompt.wav"), TEXT, None, max_text_tokens_per_sentence=12, **gen)
    assert sr == 24000 and got.dtype == np.int16 and got.shape[1] == 1
    _close(got[:, 0], want)
    out = tmp_path / "sub" / "gen.wav"
    assert fn(str(ckpt[0] / "prompt.wav"), TEXT, str(out), max_text_tokens_per_sentence=12, **gen) == str(out)
    np.testing.assert_array_equal(_read_wav(out), got[:, 0])


def test_infer_reference_defaults_run(ckpt, tts):
    """srt_dubbing calls infer(text=, audio_prompt=, output_path=None) with the reference defaults
    (beam-sample: do_sample=True, num_beams=3, top_k 30, top_p 0.8): decoded by the HIP beam kernels,
    no decoding-mode warning, reproducible for a fixed seed."""
    import warnings
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        sr, got = tts.infer(text="Mind the gap.", audio_prompt=str(ckpt[0] / "prompt.wav"), output_path=None,
                            max_mel_tokens=24, seed=1)
    assert not [w for w in rec if "num_beams" in str(w.message) or "ignored generation" in str(w.message)]
    assert sr == 24000 and got.shape[0] > 0 and got.shape[0] % 1024 == 0
    _, again = tts.infer(text="Mind the gap.", audio_prompt=str(ckpt[0] / "prompt.wav"), output_path=None,
                         max_mel_tokens=24, seed=1)
    np.testing.assert_array_equal(again, got)


# ------------------------------------------------------------------ sampling kernel
def _hf_probs(logits, temperature, top_k, top_p):
    """HF TemperatureLogitsWarper -> TopKLogitsWarper -> TopPLogitsWarper -> softmax (fp32)."""
    s = logits / temperature
    if top_k > 0:
        kth = torch.topk(s, top_k).values[..., -1, None]
        s = s.masked_fill(s < kth, float("-inf"))
    if top_p < 1.0:
        ss, si = torch.sort(s, descending=False)
        cum = ss.softmax(-1).cumsum(-1)
        rm = cum <= (1 - top_p)
        rm[..., -1:] = False
        s = s.masked_fill(rm.scatter(-1, si, rm), float("-inf"))
    return s.softmax(-1)


def _draw(logits_row, B, calls, temperature, top_k, top_p, seed0=1):
    from indextts import _hip
    lib = _hip.load()
    V = logits_row.numel()
    logits = logits_row.float().cuda().expand(B, V).contiguous()
    counts = torch.zeros(V, dtype=torch.long)
    for c in range(calls):
        seen = torch.zeros(B, V, dtype=torch.uint8, device="cuda")
        done = torch.zeros(B, dtype=torch.uint8, device="cuda")
        codes = torch.zeros(B, 1, dtype=torch.int32, device="cuda")
        t = torch.tensor([0, 0, seed0 + 7919 * c, 0], dtype=torch.int32, device="cuda")
        _hip.check(lib.itts_sample_topk_embed(
            logits.data_ptr(), V, V, seen.data_ptr(), done.data_ptr(), codes.data_ptr(), 1, t.data_ptr(), 0, 0,
            V - 1, 1.0, temperature, top_k, top_p, None, None, 2, 64, None, None, None, None, _hip.F32, B, None,
            _hip.stream_ptr()), "sample")
        counts += torch.bincount(codes.cpu().long().view(-1), minlength=V)
    return counts


@pytest.mark.parametrize("temperature,top_k,top_p", [(1.0, 30, 0.8), (0.7, 30, 0.8), (1.0, 5, 1.0),
                                                     (1.3, 64, 0.95), (1.0, 0, 1.0),
                                                     # general warper thresholds (select.h): any top_k, top-p only
                                                     (1.0, 100, 0.9), (1.0, 0, 0.7), (0.8, 1000, 1.0),
                                                     (1.0, 8194, 0.5), (1.0, 65, 1.0)])
def test_sampling_distribution(temperature, top_k, top_p):
    g = torch.Generator().manual_seed(0)
    V = 8194
    logits = torch.randn(V, generator=g) * 1.5
    logits[torch.randperm(V, generator=g)[:12]] += torch.linspace(3, 7, 12)  # a peaked head
    p = _hf_probs(logits, temperature, top_k, top_p)
    counts = _draw(logits, 512, 80, temperature, top_k, top_p)
    N = int(counts.sum())
    f = counts.double() / N
    assert int(counts[p == 0].sum()) == 0
    sig = torch.sqrt(p.double() * (1 - p.double()) / N)
    bad = (f - p.double()).abs() > 5 * sig + 2e-3
    assert not bool(bad.any()), (f[bad][:5], p[bad][:5])


def test_sampling_general_path_keeps_ties_and_top_only():
    """radix-select top_k (> 64) keeps every score tied with the k-th; top_p -> 0 keeps the top token."""
    V = 1000
    logits = torch.full((V,), -10.0)
    logits[:70] = torch.linspace(6.0, 5.0, 70)
    logits[[700, 701]] = float(logits[68])  # tied with the 69th largest (k = 69 -> 71 survivors)
    counts = _draw(logits, 256, 16, 1.0, 69, 1.0)
    assert int(counts[:69].sum() + counts[[700, 701]].sum()) == int(counts.sum())
    assert int(counts[69:700].sum()) == 0
    counts = _draw(logits, 256, 2, 1.0, 0, 1e-6)
    assert int(counts[0]) == int(counts.sum())


def test_sampling_keeps_ties_at_kth_value():
    V = 1000
    logits = torch.full((V,), -10.0)
    logits[[3, 50, 51, 52, 700]] = torch.tensor([5.0, 4.0, 4.0, 4.0, 4.0])
    counts = _draw(logits, 256, 8, 1.0, 2, 1.0)
    assert int(counts[[3, 50, 51, 52, 700]].sum()) == int(counts.sum())
    assert all(int(counts[i]) > 0 for i in (50, 51, 52, 700))


def test_engine_sampling_seeded_and_graph_equals_eager(golden):
    from indextts.gpt.engine import HipGPT
    from indextts.utils.config import tiny_config
    from indextts.utils.synthetic import gpt_state_dict
    cfg = tiny_config()
    eng = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.15), cfg.gpt, "cuda", dtype="bf16", max_kv=256)
    conds = eng.conditioning(torch.from_numpy(golden["tiny_gpt_mel"]).cuda())
    text = torch.from_numpy(golden["tiny_gpt_text"]).cuda().expand(4, -1).contiguous()
    kw = dict(do_sample=True, top_k=30, top_p=0.8, temperature=1.0, repetition_penalty=10.0)
    a = eng.generate(conds, text, 48, seed=123, use_graph=True, **kw)
    b = eng.generate(conds, text, 48, seed=123, use_graph=False, **kw)
    c = eng.generate(conds, text, 48, seed=124, use_graph=True, **kw)
    assert torch.equal(a, b)
    assert not torch.equal(a, c)
    assert not torch.equal(a[0], a[1])  # rows draw independently
    greedy = eng.generate(conds, text, 48, use_graph=True)
    assert torch.equal(greedy[0], greedy[1])


def test_infer_many_equals_infer_per_text(ckpt, tts, tmp_path):
    """long-form entry point: every text's result equals ``infer`` on it alone (greedy, f32)."""
    texts = ["Mind the gap.", TEXT, "", "Please stand clear of the closing doors."]
    gen = dict(do_sample=False, num_beams=1, max_mel_tokens=24)
    prompt = str(ckpt[0] / "prompt.wav")
    got = tts.infer_many(prompt, texts, max_text_tokens_per_sentence=12, **gen)
    assert len(got) == len(texts)
    for t, g in zip(texts, got):
        sr, want = tts.infer(prompt, t, None, max_text_tokens_per_sentence=12, **gen)
        assert g[0] == sr == 24000
        np.testing.assert_array_equal(g[1], want)
    paths = [str(tmp_path / f"c{i}.wav") for i in range(len(texts))]
    assert tts.infer_many(prompt, texts, paths, max_text_tokens_per_sentence=12, **gen) == paths
    np.testing.assert_array_equal(_read_wav(paths[1]), got[1][1][:, 0])
