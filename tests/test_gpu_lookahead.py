"""Cross-call batching behind the UNCHANGED srt_dubbing caller.

srt_dubbing's strategies loop over the cues and call ``IndexTTSEngine.synthesize(text=entry.text,
**kwargs)`` once per cue (strategies/basic_strategy.py:64-72), which calls ``IndexTTS.infer`` with
the kwargs filtered by ``inspect.signature(infer)`` (tts_engines/index_tts_engine.py:37-58, Q9).
``IndexTTS.infer`` finds the cue list in the calling frames and synthesises the next LOOKAHEAD cues
in one batched pass (``prefetch`` -> ``infer_many``); later calls take their results from it.

Checks (synthetic 12-cue SRT incl. a repeated cue and an empty one, tiny checkpoint, f32 mode):
  * deterministic decoding (greedy): every cue's int16 PCM equals the per-call result bit for bit;
  * the caller's loop issues ONE batched synthesis instead of one per cue;
  * the srt_dubbing engine/strategy code path (reproduced below verbatim in structure) runs with the
    reference's default decoding (beam sample) through the lookahead, one pass, every cue answered;
  * repeated calls for the same cue (synthesize_to_duration's retries) synthesise anew.
"""
import inspect

import numpy as np
import pytest

from test_gpu_infer import ckpt, tts  # noqa: F401  (fixtures: synthetic checkpoint, IndexTTS)

pytestmark = pytest.mark.gpu

CUES = ["Mind the gap.", "Please stand clear of the closing doors.", "There is a vehicle arriving in dock.",
        "Mind the gap.", "The next station is the last stop.", "", "Doors closing.",
        "Please take all your belongings with you.", "This train terminates here.", "Change here.",
        "Stand clear.", "Thank you for travelling with us."]
GREEDY = dict(do_sample=False, num_beams=1, max_mel_tokens=24)


class _Entry:  # srt_parser.SRTEntry: index, start_time, end_time, text
    def __init__(self, index, text):
        self.index, self.start_time, self.end_time, self.text = index, 0.5 * index, 0.5 * index + 0.4, text
        self.duration = 0.4


class _Engine:  # IndexTTSEngine (tts_engines/index_tts_engine.py:20-63), same calls
    def __init__(self, tts_model):
        self.tts_model = tts_model
        self.valid_infer_params = set(inspect.signature(self.tts_model.infer).parameters.keys())

    def synthesize(self, text, **kwargs):
        filtered = {k: v for k, v in kwargs.items() if k in self.valid_infer_params}
        sr, pcm = self.tts_model.infer(text=text, audio_prompt=kwargs["voice_reference"], output_path=None, **filtered)
        return pcm.astype(np.float32) / 32768.0, sr


def _basic_strategy(engine, entries, **kwargs):  # BasicStrategy.process_entries' loop
    segs = []
    for i, entry in enumerate(entries):
        audio, _ = engine.synthesize(text=entry.text, **kwargs)
        segs.append(audio)
    return segs


def _count_passes(tts, monkeypatch):
    calls = {"many": 0, "one": 0}
    many, one = tts.engine.synthesize_many, tts.engine.synthesize

    def _many(*a, **k):
        calls["many"] += 1
        return many(*a, **k)

    def _one(*a, **k):
        calls["one"] += 1
        return one(*a, **k)
    monkeypatch.setattr(tts.engine, "synthesize_many", _many)
    monkeypatch.setattr(tts.engine, "synthesize", _one)
    return calls


def _loop_infer(tts, prompt, entries):
    out = []
    for i, entry in enumerate(entries):
        out.append(tts.infer(prompt, entry.text, None, max_text_tokens_per_sentence=12, **GREEDY)[1])
    return out


def test_lookahead_results_equal_per_call_results(ckpt, tts, monkeypatch):  # noqa: F811
    prompt = str(ckpt[0] / "prompt.wav")
    entries = [_Entry(i + 1, t) for i, t in enumerate(CUES)]
    monkeypatch.setattr(type(tts), "LOOKAHEAD", 0)
    want = _loop_infer(tts, prompt, entries)
    monkeypatch.setattr(type(tts), "LOOKAHEAD", 64)
    calls = _count_passes(tts, monkeypatch)
    got = _loop_infer(tts, prompt, entries)
    assert calls == {"many": 1, "one": 0}, calls
    for i, (g, w) in enumerate(zip(got, want)):
        np.testing.assert_array_equal(g, w, err_msg=f"cue {i}")
    assert not tts._ahead, "every prefetched result was consumed"


def test_unchanged_srt_dubbing_path_batches(ckpt, tts, monkeypatch):  # noqa: F811
    prompt = str(ckpt[0] / "prompt.wav")
    entries = [_Entry(i + 1, t) for i, t in enumerate(CUES)]
    monkeypatch.setattr(type(tts), "LOOKAHEAD", 64)
    calls = _count_passes(tts, monkeypatch)
    segs = _basic_strategy(_Engine(tts), entries, voice_reference=prompt, verbose=False)
    assert calls["many"] == 1 and calls["one"] == 0, calls
    assert len(segs) == len(CUES)
    for t, s in zip(CUES, segs):
        assert s.dtype == np.float32 and (s.size > 0) == (t != "")
    # a retry of the same cue (synthesize_to_duration's search) is a new synthesis, not the cached one
    segs2 = _basic_strategy(_Engine(tts), entries[:1], voice_reference=prompt)
    assert calls["many"] + calls["one"] >= 2
    assert segs2[0].size > 0


def test_no_cue_list_no_lookahead(ckpt, tts, monkeypatch):  # noqa: F811
    prompt = str(ckpt[0] / "prompt.wav")
    monkeypatch.setattr(type(tts), "LOOKAHEAD", 64)
    calls = _count_passes(tts, monkeypatch)
    sr, pcm = tts.infer(prompt, CUES[0], None, max_text_tokens_per_sentence=12, **GREEDY)
    assert calls == {"many": 0, "one": 1} and sr == 24000 and pcm.size > 0
