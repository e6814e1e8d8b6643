"""The persistent decode layer (csrc/gpt_layer.hip, itts_gpt_decode_steps_pl) against the launch chain
(itts_gpt_decode_steps) at the full IndexTTS-1.5 size: every layer's phases reproduce the chain
kernels' arithmetic in the same order, so the two paths must agree BIT FOR BIT -- the raw f32 logits of
every teacher-forced step and the chosen ids -- at 32 rows (C3), 1 row (C2), 128 rows (the long-form
chunks, 4 row tiles), ragged 7- and 45-row batches with left padding, and beam search / beam sample
(96 rows through the KV lineage table), with keys from the prompt block up to KV length ~160.  Parity of the chain
itself with the reference is tests/test_gpu_fullsize.py (which runs on whichever path the engine
picks: the persistent one for <= 128 rows).

Round 5: the same bit identity at the bench's own decode shape (C3: L = 48 text ids, 400 steps, keys up to
483: four 128-key rounds, the peeled round 0 and the full-depth key loop) at B = 32 and B = 1; lane reuse
with no per-step reset (epoch-tagged hand-offs); the hand-off timeout when another grid holds CUs, and the
launch-chain re-run that recovers from it; the long-form driver's tail chunk beside the back stream."""
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
_cache = {}


def _engine(max_kv=256):
    key = ("eng", max_kv)
    if key not in _cache:
        import os
        from indextts.gpt.engine import HipGPT
        from indextts.utils.config import default_config_path, load_config
        from indextts.utils.synthetic import gpt_state_dict
        cfg = load_config(default_config_path())
        old = os.environ.get("ITTS_PL")
        os.environ["ITTS_PL"] = "1"  # this engine packs the persistent-layer operands whatever the default
        try:
            _cache.clear()  # one full-size engine alive at a time
            torch.cuda.empty_cache()
            _cache[key] = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.08), cfg.gpt, "cuda", dtype="bf16", max_kv=max_kv)
            _cache[key].PL_MAX_ROWS = 128  # every shape the kernel supports, whatever the product threshold
        finally:
            if old is None:
                del os.environ["ITTS_PL"]
            else:
                os.environ["ITTS_PL"] = old
    return _cache[key]


def _run(eng, pl, conds, text, forced, n):
    eng.pl = pl
    for k in list(eng._lanes):  # fresh states / graphs per path
        del eng._lanes[k]
    eng.logits_trace = []
    try:
        codes = eng.generate(conds, text, n, min_new_tokens=n, forced_codes=forced).cpu()
        trace = torch.stack([t.cpu() for t in eng.logits_trace])
    finally:
        eng.logits_trace = None
        eng.pl = True
    return codes, trace


@pytest.mark.parametrize("B", [32, 1, 7, 128, 45])
def test_persistent_layer_bit_identical_to_launch_chain(B):
    eng = _engine()
    if not eng.pl or not eng._pl_ok({"B": B}):
        pytest.skip("persistent layer not available on this device")
    g = torch.Generator().manual_seed(40 + B)
    L = 24
    lens = [L] * B if B not in (7, 45) else [(24, 5, 17, 24, 9, 1, 20)[i % 7] for i in range(B)]  # ragged
    text = torch.stack([torch.nn.functional.pad(torch.randint(2, 12000, (n,), generator=g), (0, L - n), value=1)
                        for n in lens]).cuda()
    conds = torch.randn(B, 32, 1024, generator=g).cuda()
    n = 96
    forced = torch.randint(0, 8192, (B, n), generator=g).cuda()
    c_pl, t_pl = _run(eng, True, conds, text, forced, n)
    c_ch, t_ch = _run(eng, False, conds, text, forced, n)
    assert torch.isfinite(t_pl).all()
    assert torch.equal(c_pl, c_ch)
    bad = (t_pl != t_ch).nonzero()
    assert bad.numel() == 0, (bad[:5], t_pl[tuple(bad[0])] if bad.numel() else None)
    assert eng.pl_error() == 0


def test_persistent_layer_free_running_equals_chain():
    """free-running greedy decode (ids fed back) at C3's shape: same ids on both paths"""
    eng = _engine()
    if not eng.pl or not eng._pl_ok({"B": 32}):
        pytest.skip("persistent layer not available on this device")
    g = torch.Generator().manual_seed(77)
    text = torch.randint(2, 12000, (32, 40), generator=g).cuda()
    conds = torch.randn(32, 32, 1024, generator=g).cuda()
    outs = []
    for pl in (True, False):
        eng.pl = pl
        for k in list(eng._lanes):
            del eng._lanes[k]
        outs.append(eng.generate(conds, text, 120, min_new_tokens=120).cpu())
    eng.pl = True
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("do_sample", [False, True])
@pytest.mark.parametrize("nutt", [32, 10, 21])
def test_persistent_layer_beams_equal_chain(do_sample, nutt):
    """beam search / beam sample (3 beams x 32 / 10 / 21 utterances = 96 / 30 / 63 rows: one to three row tiles,
    keys through the lineage table; the beam-major attention, one pass over each utterance's beams) on the
    persistent layers: the same hypotheses as on the launch chain; ragged text lengths (left padding) for 10 / 21"""
    eng = _engine()
    if not eng.pl or not eng._pl_ok({"B": 3 * nutt, "kv_rows": True}):
        pytest.skip("persistent layer not available on this device")
    g = torch.Generator().manual_seed(91 + nutt)
    L = 30
    lens = [L] * nutt if nutt == 32 else [int(torch.randint(5, L + 1, (1,), generator=g)) for _ in range(nutt)]
    text = torch.stack([torch.nn.functional.pad(torch.randint(2, 12000, (n,), generator=g), (0, L - n), value=1)
                        for n in lens]).cuda()
    conds = torch.randn(nutt, 32, 1024, generator=g).cuda()
    outs = []
    for pl in (True, False):
        eng.pl = pl
        for k in list(eng._lanes):
            del eng._lanes[k]
        outs.append(eng.generate(conds, text, 80, num_beams=3, do_sample=do_sample, top_k=30, top_p=0.8,
                                 seed=7).cpu())
    eng.pl = True
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B", [32, 1])
def test_persistent_layer_bit_identical_at_c3_decode_shape(B):
    """C3's decode as bench.py runs it: L = 48 text ids (s + 1 = 83 keys of prompt block), 400 teacher-forced
    steps (keys up to 483), raw logits of every step and the chosen ids bit-identical to the launch chain"""
    eng = _engine(max_kv=600)
    if not eng.pl or not eng._pl_ok({"B": B}):
        pytest.skip("persistent layer not available on this device")
    g = torch.Generator().manual_seed(500 + B)
    text = torch.randint(2, 12000, (B, 48), generator=g).cuda()
    conds = torch.randn(B, 32, 1024, generator=g).cuda()
    n = 400
    forced = torch.randint(0, 8192, (B, n), generator=g).cuda()
    c_pl, t_pl = _run(eng, True, conds, text, forced, n)
    c_ch, t_ch = _run(eng, False, conds, text, forced, n)
    assert t_pl.shape[0] == n and torch.isfinite(t_pl).all()
    assert torch.equal(c_pl, c_ch)
    bad = (t_pl != t_ch).nonzero()
    assert bad.numel() == 0, (bad[:5], t_pl[tuple(bad[0])] if bad.numel() else None)
    assert eng.pl_error() == 0


def test_persistent_layer_lane_reuse_without_reset():
    """four generate calls on one kept lane (same shape: the state and the captured graph are reused, the
    epoch keeps growing and nothing is reset between calls or steps), different inputs each time: every
    call's ids equal a fresh chain run's"""
    eng = _engine()
    if not eng.pl or not eng._pl_ok({"B": 32}):
        pytest.skip("persistent layer not available on this device")
    for k in list(eng._lanes):
        del eng._lanes[k]
    got, want = [], []
    for i in range(4):
        g = torch.Generator().manual_seed(900 + i)
        text = torch.randint(2, 12000, (32, 24), generator=g).cuda()
        conds = torch.randn(32, 32, 1024, generator=g).cuda()
        eng.pl = True
        got.append(eng.generate(conds, text, 64, min_new_tokens=64).cpu())
        assert eng._pl_ran and eng.pl_error() == 0
        with eng.launch_chain():
            want.append(eng.generate(conds, text, 64, min_new_tokens=64).cpu())
        assert not eng._pl_ran
    for a, b in zip(got, want):
        assert torch.equal(a, b)


def test_persistent_layer_timeout_reruns_on_chain():
    """another grid holding 128 CUs for 1.5 s (itts_diag_occupy, one 120-KiB-LDS workgroup per CU) while the
    persistent decode starts: its resident workgroups time out (no hang), the error word is set, the engine
    re-arms the scratch and re-runs the call on the launch chain -- ids identical to an undisturbed run --
    and the next call runs on the persistent layers again"""
    from indextts import _hip
    eng = _engine()
    if not eng.pl or not eng._pl_ok({"B": 32}):
        pytest.skip("persistent layer not available on this device")
    g = torch.Generator().manual_seed(4242)
    text = torch.randint(2, 12000, (32, 24), generator=g).cuda()
    conds = torch.randn(32, 32, 1024, generator=g).cuda()
    want = eng.generate(conds, text, 24, min_new_tokens=24).cpu()
    assert eng.pl_error() == 0
    strikes = eng._pl_strikes
    # a side stream may share its hardware queue with the decode lane's (HIP maps streams onto
    # GPU_MAX_HW_QUEUES = 4 queues round-robin): then the occupier simply runs first, nothing is concurrent and
    # the decode cannot time out -- its ids must still be right; a fresh stream is tried (up to 4)
    timed_out = False
    for attempt in range(4):
        side = torch.cuda.Stream(priority=-1) if attempt == 0 else torch.cuda.Stream()
        sink = torch.zeros(128, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        _hip.check(eng.lib.itts_diag_occupy(128, 1_500_000, sink.data_ptr(), side.cuda_stream), "itts_diag_occupy")
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            got = eng.generate(conds, text, 24, min_new_tokens=24).cpu()
        torch.cuda.synchronize()
        assert int(sink.sum()) == 128 * 63  # the occupying workgroups ran and exited
        assert torch.equal(got, want)
        if any("hand-off timeout" in str(w.message) for w in rec):
            timed_out = True
            break
        assert eng._pl_ran and eng.pl_error() == 0
    if not timed_out:
        pytest.skip("the occupying grid never ran beside the decode (shared hardware queue); ids checked")
    assert eng._pl_strikes == strikes + 1 and eng.pl
    assert torch.equal(got, want)
    assert eng.pl_error() == 0  # re-armed
    again = eng.generate(conds, text, 24, min_new_tokens=24).cpu()
    assert eng._pl_ran and eng.pl_error() == 0 and torch.equal(again, want)
    eng._pl_strikes = strikes


def test_synthesize_many_tail_chunk_beside_back_stream():
    """the long-form driver's shape: a 128-row chunk then a 20-row tail chunk through synthesize_many (the
    tail's decode overlaps the first chunk's latent pass + vocoder on the back stream, so it runs on the
    launch chain), equal to serial synthesize per chunk (whose 20-row decode runs on the persistent layers),
    with no hand-off error"""
    from indextts.pipeline import BatchedTTS
    from indextts.utils.config import default_config_path, load_config
    from indextts.utils.synthetic import bigvgan_state_dict, gpt_state_dict
    import os
    _cache.clear()
    torch.cuda.empty_cache()
    cfg = load_config(default_config_path())
    old = os.environ.get("ITTS_PL")
    os.environ["ITTS_PL"] = "1"
    try:
        tts = BatchedTTS(gpt_state_dict(cfg.gpt, 0, 0.08), bigvgan_state_dict(cfg.bigvgan, 0), cfg, "cuda", "bf16",
                         max_kv=256)
    finally:
        if old is None:
            del os.environ["ITTS_PL"]
        else:
            os.environ["ITTS_PL"] = old
    if not tts.gpt.pl or not tts.gpt._pl_ok({"B": 20}):
        pytest.skip("persistent layer not available on this device")
    rng = np.random.default_rng(17)

    def batch(n):
        mels = [torch.from_numpy(rng.normal(-4, 2, (1, 100, 80)).astype(np.float32)).cuda() for _ in range(n)]
        texts = [torch.from_numpy(rng.integers(2, 12000, int(rng.integers(8, 30)))).cuda() for _ in range(n)]
        return mels, texts

    batches = [batch(128), batch(20)]
    want = []
    for m, t in batches:
        want.append(tts.synthesize(m, t, max_mel_tokens=24, min_new_tokens=24))
        assert tts.gpt._pl_ran == tts.gpt.pl_takes(len(t))
    # overlap forced: auto would run these batches back to back when every chunk fits the persistent layers
    got = tts.synthesize_many(batches, max_mel_tokens=24, min_new_tokens=24, overlap=True)
    torch.cuda.synchronize()
    assert not tts.gpt._pl_ran  # the tail chunk beside the back stream: launch chain
    assert tts.gpt.pl_error() == 0
    for w, g in zip(want, got):
        assert torch.equal(w[1], g[1])
        assert all(torch.equal(x, y) for x, y in zip(w[2], g[2]))
        for i in range(len(w[1])):
            n = int(w[1][i])
            assert torch.equal(w[0][i, :n], g[0][i, :n]), i
