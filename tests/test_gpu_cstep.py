"""The whole decode step as one C-ABI call (``itts_gpt_decode_step``, csrc/gpt_step.hip) against the
Python launch sequence of the bf16 product path (``HipGPT._decode_step_fold``): the same kernels,
launched from C++.  Bar: the raw f32 logits of EVERY step are bit-identical, and so are the ids
(greedy, top-k/top-p sampling with a fixed seed, beam search / beam sample).  Cases: tiny and full IndexTTS-1.5 size, left-padded batches (L ~ U[16, 96] at full size),
B = 32 (the C3 shape), KV lengths past one attention round (> 320 keys), beams (R = 24 rows).
The reference parity of the per-kernel path itself is tests/test_gpu_fullsize.py.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
_cache = {}


def _engine(size):
    if size not in _cache:
        from indextts.gpt.engine import HipGPT
        from indextts.utils.config import default_config_path, load_config, tiny_config
        from indextts.utils.synthetic import gpt_state_dict
        cfg = tiny_config() if size == "tiny" else load_config(default_config_path())
        sd = gpt_state_dict(cfg.gpt, 0, 0.08)
        _cache[size] = HipGPT(sd, cfg.gpt, "cuda", dtype="bf16")
    return _cache[size]


def _inputs(eng, B, lmin, lmax, seed):
    g = torch.Generator().manual_seed(seed)
    L = lmax
    conds = torch.randn(B, 32, eng.D, generator=g)
    text = torch.randint(2, 6000, (B, L), generator=g)
    for b in range(B):  # left-pad the shorter rows with the stop id (stripped by prepare_gpt_inputs, Q3)
        n = int(torch.randint(lmin, lmax + 1, (1,), generator=g))
        text[b, : L - n] = 1
    return conds.cuda(), text.cuda()


def _run(eng, cstep, conds, text, steps, **kw):
    eng.cstep = cstep
    eng.logits_trace = [] if kw.get("num_beams", 1) == 1 else None
    try:
        codes = eng.generate(conds, text, steps, **kw)
        torch.cuda.synchronize()
        tr = None if eng.logits_trace is None else torch.stack(eng.logits_trace).cpu()
    finally:
        eng.logits_trace = None
        eng.cstep = True
    return codes.cpu(), tr


@pytest.mark.parametrize("size,B,lmin,lmax,steps", [("tiny", 5, 3, 12, 40), ("full", 32, 16, 96, 48),
                                                     ("full", 3, 90, 96, 300)])
def test_step_greedy_bit_identical(size, B, lmin, lmax, steps):
    eng = _engine(size)
    conds, text = _inputs(eng, B, lmin, lmax, 11 + B)
    kw = dict(min_new_tokens=steps, repetition_penalty=10.0)
    c0, t0 = _run(eng, False, conds, text, steps, **kw)
    c1, t1 = _run(eng, True, conds, text, steps, **kw)
    assert t0.shape == t1.shape
    diff = (t0 != t1).any(-1).any(-1)
    assert not bool(diff.any()), f"logits differ from step {int(diff.int().argmax())}"
    assert torch.equal(c0, c1)


def test_step_sampling_same_draws():
    eng = _engine("full")
    conds, text = _inputs(eng, 8, 16, 64, 5)
    kw = dict(min_new_tokens=0, do_sample=True, top_k=30, top_p=0.8, temperature=1.0, seed=1234)
    c0, t0 = _run(eng, False, conds, text, 40, **kw)
    c1, t1 = _run(eng, True, conds, text, 40, **kw)
    assert torch.equal(t0, t1)
    assert torch.equal(c0, c1)


@pytest.mark.parametrize("do_sample", [False, True])
def test_step_beams_same_hypotheses(do_sample):
    eng = _engine("full")
    conds, text = _inputs(eng, 8, 16, 64, 7)
    kw = dict(num_beams=3, min_new_tokens=8, do_sample=do_sample, top_k=30, top_p=0.8, seed=99)
    c0, _ = _run(eng, False, conds, text, 32, **kw)
    c1, _ = _run(eng, True, conds, text, 32, **kw)
    assert torch.equal(c0, c1)


@pytest.mark.parametrize("sample", [False, True])
def test_multi_step_call_equals_single_steps(sample, monkeypatch):
    """itts_gpt_decode_steps (4 steps per captured graph, one counter advance) vs one-step graph
    replays of itts_gpt_decode_step: identical ids / draws over 50 steps (several 4-step replays,
    the done-check boundaries, and the single-step tail)."""
    from indextts.gpt.engine import HipGPT
    eng = _engine("full")
    conds, text = _inputs(eng, 32, 16, 96, 3)
    kw = dict(min_new_tokens=50, repetition_penalty=10.0)
    if sample:
        kw.update(do_sample=True, top_k=30, top_p=0.8, seed=77)
    monkeypatch.setattr(HipGPT, "GRAPH_STEPS", 1)
    c1 = eng.generate(conds, text, 50, **kw).cpu()
    monkeypatch.setattr(HipGPT, "GRAPH_STEPS", 4)
    for ln in eng._lanes.values():
        if isinstance(ln, dict):
            HipGPT._drop_graphs(ln)
    c4 = eng.generate(conds, text, 50, **kw).cpu()
    assert torch.equal(c1, c4)
