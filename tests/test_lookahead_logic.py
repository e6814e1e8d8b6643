"""CPU tests of the cross-call batching control logic of ``IndexTTS.infer`` (indextts/infer.py) and of
the multi-GPU worker protocol (indextts/devpool.py), with a fake synthesis underneath (stub_tts).

The caller loops are the reference's: srt_dubbing's strategies call ``IndexTTSEngine.synthesize``
once per cue (srt_dubbing/src/strategies/basic_strategy.py:65-74); ``synthesize_to_duration``
retries one cue up to 5 times with a binary-searched ``length_penalty``
(tts_engines/index_tts_engine.py:65-107; IndexTTSEngine filters it out by ``inspect.signature``
(quirk Q9), a caller that passes it straight to ``infer`` does not).  Checked:
  * every cue gets exactly its own result, in order, from ONE batched pass per window;
  * a loop whose variables are not named ``entries`` / ``i`` is batched too;
  * a duration search that varies the arguments per attempt costs one single call per attempt (never
    a window per attempt), and the prefetched store stays bounded;
  * one failing cue fails only itself (the strategies turn that into silence), not its window;
  * the worker protocol: results dealt over workers come back in order; a worker error or death
    falls back to this process; a worker that cannot start is skipped.
"""
import numpy as np
import pytest

from indextts.devpool import DevicePool, deal, parse_devices
from stub_tts import POISON, StubTTS, fake_pcm

PROMPT = "/nonexistent/prompt.wav"  # a path: lookahead keys use it (mtime None)
CUES = [f"cue number {i} " + "word " * (i % 5) for i in range(11)]


class _Entry:
    def __init__(self, i, text):
        self.index, self.text, self.duration = i, text, 0.4


def _basic(tts, entries, **kw):  # BasicStrategy.process_entries' loop (silence on error)
    out = []
    for i, entry in enumerate(entries):
        try:
            out.append(tts.infer(PROMPT, entry.text, None, **kw)[1])
        except ValueError:
            out.append(None)
    return out


def _renamed(tts, cues, **kw):  # same loop, other variable names
    got = []
    for k, cue in enumerate(cues):
        got.append(tts.infer(PROMPT, cue.text, None, **kw)[1])
    return got


def test_window_batches_and_results_in_order():
    tts = StubTTS()
    tts.LOOKAHEAD = 64
    entries = [_Entry(i, t) for i, t in enumerate(CUES)]
    got = _basic(tts, entries, do_sample=False)
    assert [c[0] for c in tts.calls] == ["many"]
    for t, g in zip(CUES, got):
        np.testing.assert_array_equal(g, fake_pcm(t, {"do_sample": False}))
    assert not tts._ahead


def test_renamed_loop_variables_are_batched():
    tts = StubTTS()
    tts.LOOKAHEAD = 64
    cues = [_Entry(i, t) for i, t in enumerate(CUES)]
    got = _renamed(tts, cues)
    assert [c[0] for c in tts.calls] == ["many"]
    for t, g in zip(CUES, got):
        np.testing.assert_array_equal(g, fake_pcm(t, {}))


def test_no_list_no_lookahead_and_pathless_prompt():
    tts = StubTTS()
    tts.LOOKAHEAD = 64
    tts.infer(PROMPT, CUES[0], None)
    tts.infer(object(), CUES[1], None)  # not a path: never cached across calls
    assert [c[0] for c in tts.calls] == ["one", "one"]


def test_windows_advance_and_store_is_bounded():
    tts = StubTTS()
    tts.LOOKAHEAD = 4
    entries = [_Entry(i, t) for i, t in enumerate(CUES)]
    got = _basic(tts, entries)
    assert [c[0] for c in tts.calls] == ["many", "many", "many"]  # 11 cues, windows of 4
    assert [len(c[1]) for c in tts.calls] == [4, 4, 3]
    for t, g in zip(CUES, got):
        np.testing.assert_array_equal(g, fake_pcm(t, {}))
    assert sum(len(q) for q in tts._ahead.values()) == 0


def _duration_search(tts, text, direct):
    """IndexTTSEngine.synthesize_to_duration: 5 attempts, penalty bisected in [-2, 2]."""
    lo, hi = -2.0, 2.0
    for attempt in range(5):
        pen = (lo + hi) / 2
        kw = {"length_penalty": pen} if direct else {}
        tts.infer(PROMPT, text, None, **kw)
        hi = pen if attempt % 2 else hi
        lo = lo if attempt % 2 else pen


@pytest.mark.parametrize("direct", [False, True])
def test_duration_search_costs_no_extra_windows(direct):
    tts = StubTTS()
    tts.LOOKAHEAD = 64
    entries = [_Entry(i, t) for i, t in enumerate(CUES)]
    for i, entry in enumerate(entries):  # AdaptiveStrategy's loop
        _duration_search(tts, entry.text, direct)
    texts = [len(c[1]) if c[0] == "many" else 1 for c in tts.calls]
    # one window of every cue; then each retry synthesises that cue alone (filtered kwargs, Q9: the
    # retry repeats the first attempt's arguments; a direct caller's new penalty: one call per attempt)
    assert texts[0] == len(CUES) and all(n == 1 for n in texts[1:])
    assert sum(texts) == len(CUES) + 4 * len(CUES)
    assert sum(len(q) for q in tts._ahead.values()) <= len(CUES)


def test_unused_windows_switch_the_lookahead_off():
    tts = StubTTS()
    tts.LOOKAHEAD = 8
    texts = [f"line {i}" for i in range(40)]
    entries = [_Entry(i, t) for i, t in enumerate(texts)]
    for i, entry in enumerate(entries):  # a caller that changes max tokens on every cue
        tts.infer(PROMPT, entry.text, None, max_text_tokens_per_sentence=100 + i)
    many = [c for c in tts.calls if c[0] == "many"]
    assert len(many) == 3, len(many)  # three mostly-unused windows, then one call per cue


def test_poisoned_cue_fails_alone():
    tts = StubTTS()
    tts.LOOKAHEAD = 64
    texts = list(CUES)
    texts[5] = POISON
    entries = [_Entry(i, t) for i, t in enumerate(texts)]
    with pytest.warns(RuntimeWarning, match="lookahead batch"):
        got = _basic(tts, entries)
    assert [g is None for g in got] == [i == 5 for i in range(len(texts))]
    for i, (t, g) in enumerate(zip(texts, got)):
        if i != 5:
            np.testing.assert_array_equal(g, fake_pcm(t, {}))
    assert sum(c[0] == "many" for c in tts.calls) == 1  # the failed window is not retried


def test_deal_and_parse_devices():
    bins = deal([5, 1, 9, 3, 3, 7], 3)
    assert sorted(i for b in bins for i in b) == list(range(6))
    loads = [sum([5, 1, 9, 3, 3, 7][i] for i in b) for b in bins]
    assert max(loads) - min(loads) <= 2
    assert parse_devices("", 8) == [] and parse_devices(None, 8) == []
    assert parse_devices("all", 2) == ["cuda:0", "cuda:1"]
    assert parse_devices("0, 0,cuda:1", 2) == ["cuda:0", "cuda:0", "cuda:1"]
    with pytest.raises(ValueError):
        parse_devices("3", 2)


def test_device_pool_protocol_spawned_workers():
    pool = DevicePool("cfg", "dir", True, ["cuda:1", "cuda:7", "cuda:2"], builder="stub_tts:WorkerStub")
    try:
        assert pool.alive() == [0, 2]  # cuda:7's worker failed to start and is skipped
        tts = StubTTS(pool=pool)
        tts.LOOKAHEAD = 64
        entries = [_Entry(i, t) for i, t in enumerate(CUES)]
        got = _basic(tts, entries, do_sample=False)
        for t, g in zip(CUES, got):
            np.testing.assert_array_equal(g, fake_pcm(t, {"do_sample": False}))
        local = [c for c in tts.calls if c[0] == "many"]
        assert len(local) == 1 and 0 < len(local[0][1]) < len(CUES)  # this process took one share of three
        # a worker error: its share is redone here, results still exact
        texts = ["a " * 20, POISON, "x"]  # longest first: the poisoned cue lands on a worker
        with pytest.warns(RuntimeWarning, match="poisoned"):
            with pytest.raises(ValueError):
                tts._infer_many_devices(PROMPT, texts, 120, {})
        texts = [f"other {i}" for i in range(6)]
        res = tts._infer_many_devices(PROMPT, texts, 120, {})
        for t, r in zip(texts, res):
            np.testing.assert_array_equal(r[1], fake_pcm(t, {}))
        # a worker dies mid-request: dropped, its share redone here
        with pytest.warns(RuntimeWarning, match="died"):
            res = tts._infer_many_devices(PROMPT, ["__die__", "a b c d e f g h", "x", "y y"], 120, {})
        assert len(pool.alive()) == 1
    finally:
        pool.close()


def test_device_pool_hung_and_out_of_step_workers_are_dropped():
    """a worker that does not answer within the request timeout is terminated and its
    share redone locally; a reply for another request id (the pipe out of step) kills the worker
    instead of poisoning every later share."""
    pool = DevicePool("cfg", "dir", True, ["cuda:1", "cuda:2"], builder="stub_tts:WorkerStub")
    try:
        assert pool.alive() == [0, 1]
        pool.request_timeout = 3.0
        tts = StubTTS(pool=pool)
        texts = ["a " * 20, "__hang__ " * 8, "x", "y y"]  # longest first: the hanging cue lands on a worker
        with pytest.warns(RuntimeWarning, match="no reply"):
            res = tts._infer_many_devices(PROMPT, texts, 120, {})
        for t, r in zip(texts, res):
            np.testing.assert_array_equal(r[1], fake_pcm(t, {}))
        assert len(pool.alive()) == 1
        # out of step: request A's reply is never collected, request B then reads A's reply
        wi = pool.alive()[0]
        pool.submit(wi, PROMPT, ["a"], 120, {})
        tb = pool.submit(wi, PROMPT, ["b"], 120, {})
        from indextts.devpool import WorkerError
        with pytest.raises(WorkerError, match="reply"):
            pool.result(tb)
        assert pool.alive() == []
    finally:
        pool.close()
