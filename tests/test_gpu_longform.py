"""Long-form serving behind the UNCHANGED srt_dubbing caller at full IndexTTS-1.5 size, bf16 (what
srt_dubbing's ``IndexTTSConfig`` runs: ``is_fp16=True``; SURVEY.md §8(f)3, BASELINE.json configs[4]).

srt_dubbing's strategies call ``IndexTTSEngine.synthesize`` -> ``infer`` once per cue
(srt_dubbing/src/strategies/basic_strategy.py:65-74 -> tts_engines/index_tts_engine.py:45-63; the
whole engine/strategy structure runs in test_gpu_lookahead.py).
Synthetic full-size checkpoint (seeded weights, the reference's directory layout), greedy decoding:
  * the cue lookahead (one batched pass for the cue list) gives every cue the int16 PCM of its own
    per-call synthesis, bit for bit;
  * with ``ITTS_DEVICES=0,0`` (one spawned worker process beside this process's engine, both on the
    box's one GPU: the stand-in for two GPUs) every cue's PCM is again bit-identical, and the work was
    really dealt over both engines.
"""
import numpy as np
import pytest

from test_gpu_lookahead import _Entry

pytestmark = pytest.mark.gpu

CUES = ["Mind the gap.", "Please stand clear of the closing doors.", "There is a vehicle arriving in dock.",
        "Mind the gap.", "The next station is the last stop.", "Doors closing.",
        "Please take all your belongings with you.", "Change here for the northern line."]
GREEDY = dict(do_sample=False, num_beams=1, max_mel_tokens=40)


@pytest.fixture(scope="module")
def full_ckpt(tmp_path_factory):
    import os
    from indextts.utils.config import default_config_path, load_config
    from indextts.utils.synthetic import write_checkpoint_dir
    d = tmp_path_factory.mktemp("ckpt_full")
    here = os.path.dirname(os.path.abspath(__file__))
    cfg_path = write_checkpoint_dir(str(d), load_config(default_config_path()),
                                    os.path.join(here, "golden", "tiny_bpe.model"), seed=0, mel_head_std=0.08)
    _write_prompt(d / "prompt.wav")
    return d, cfg_path


def _write_prompt(path):
    import wave
    sr, n = 16000, 48000
    tt = np.arange(n) / sr
    rng = np.random.default_rng(1)
    sig = 0.3 * np.sin(2 * np.pi * (120 + 150 * tt) * tt) + 0.05 * rng.standard_normal(n)
    pcm = (np.stack([sig, 0.7 * sig], 1) * 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm.tobytes())


@pytest.fixture(scope="module")
def per_call(full_ckpt):
    """Each cue synthesised by its own infer call (no lookahead), on a single-device IndexTTS."""
    import os
    from indextts.infer import IndexTTS
    d, cfg_path = full_ckpt
    old = os.environ.pop("ITTS_DEVICES", None)
    tts = IndexTTS(cfg_path=cfg_path, model_dir=str(d), is_fp16=True, device="cuda:0")
    if old is not None:
        os.environ["ITTS_DEVICES"] = old
    tts.LOOKAHEAD = 0
    want = [tts.infer(str(d / "prompt.wav"), t, None, **GREEDY)[1] for t in CUES]
    return tts, want


def _srt_run(tts, d):
    """BasicStrategy's cue loop calling infer directly with greedy decoding (through IndexTTSEngine the
    decoding kwargs would be filtered out by its inspect.signature check, Q9, leaving the reference's
    default beam sampling, whose draws are random)."""
    entries = [_Entry(i + 1, t) for i, t in enumerate(CUES)]
    out = []
    for i, entry in enumerate(entries):
        out.append(tts.infer(str(d / "prompt.wav"), entry.text, None, **GREEDY)[1])
    return out


def test_full_size_bf16_lookahead_equals_per_call(full_ckpt, per_call, monkeypatch):
    d, _ = full_ckpt
    tts, want = per_call
    monkeypatch.setattr(tts, "LOOKAHEAD", 128)
    calls = {"many": 0}
    many = tts.engine.synthesize_many

    def _many(*a, **k):
        calls["many"] += 1
        return many(*a, **k)
    monkeypatch.setattr(tts.engine, "synthesize_many", _many)
    got = _srt_run(tts, d)
    assert calls["many"] == 1
    assert all(w.size > 0 for w in want)
    for i, (g, w) in enumerate(zip(got, want)):
        np.testing.assert_array_equal(g, w, err_msg=f"cue {i}")


def test_two_engines_one_gpu_equal_per_call(full_ckpt, per_call, monkeypatch):
    from indextts.infer import IndexTTS
    d, cfg_path = full_ckpt
    _, want = per_call
    monkeypatch.setenv("ITTS_DEVICES", "0,0")
    tts = IndexTTS(cfg_path=cfg_path, model_dir=str(d), is_fp16=True, device="cuda:0")
    try:
        assert tts.n_devices == 2, "the worker process did not start"
        tts.LOOKAHEAD = 128
        local = []
        many = tts.infer_many

        def _many(prompt, texts, *a, **k):
            local.append(list(texts))
            return many(prompt, texts, *a, **k)
        monkeypatch.setattr(tts, "infer_many", _many)
        got = _srt_run(tts, d)
        assert len(local) == 1 and 0 < len(local[0]) < len(CUES), local  # the worker took the rest
        for i, (g, w) in enumerate(zip(got, want)):
            np.testing.assert_array_equal(g, w, err_msg=f"cue {i}")
    finally:
        tts.close()
