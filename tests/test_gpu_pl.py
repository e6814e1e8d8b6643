"""The persistent decode layer (csrc/gpt_layer.hip, itts_gpt_decode_steps_pl) against the launch chain
(itts_gpt_decode_steps) at the full IndexTTS-1.5 size: every layer's phases reproduce the chain
kernels' arithmetic in the same order, so the two paths must agree BIT FOR BIT -- the raw f32 logits of
every teacher-forced step and the chosen ids -- at 32 rows (C3), 1 row (C2), 128 rows (the long-form
chunks, 4 row tiles), ragged 7- and 45-row batches with left padding, and beam search / beam sample
(96 rows through the KV lineage table), with keys from the prompt block up to KV length ~160.  Parity of the chain
itself with the reference is tests/test_gpu_fullsize.py (which runs on whichever path the engine
picks: the persistent one for <= 32 rows)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
_cache = {}


def _engine():
    if "eng" not in _cache:
        import os
        from indextts.gpt.engine import HipGPT
        from indextts.utils.config import default_config_path, load_config
        from indextts.utils.synthetic import gpt_state_dict
        cfg = load_config(default_config_path())
        old = os.environ.get("ITTS_PL")
        os.environ["ITTS_PL"] = "1"  # this engine packs the persistent-layer operands whatever the default
        try:
            _cache["eng"] = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.08), cfg.gpt, "cuda", dtype="bf16", max_kv=256)
            _cache["eng"].PL_MAX_ROWS = 128  # every shape the kernel supports, whatever the product threshold
        finally:
            if old is None:
                del os.environ["ITTS_PL"]
            else:
                os.environ["ITTS_PL"] = old
    return _cache["eng"]


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
def test_persistent_layer_beams_equal_chain(do_sample):
    """beam search / beam sample (3 beams x 32 utterances = 96 rows, keys through the lineage table) on the
    persistent layers: the same hypotheses as on the launch chain"""
    eng = _engine()
    if not eng.pl or not eng._pl_ok({"B": 96}):
        pytest.skip("persistent layer not available on this device")
    g = torch.Generator().manual_seed(91)
    text = torch.randint(2, 12000, (32, 30), generator=g).cuda()
    conds = torch.randn(32, 32, 1024, generator=g).cuda()
    outs = []
    for pl in (True, False):
        eng.pl = pl
        for k in list(eng._lanes):
            del eng._lanes[k]
        outs.append(eng.generate(conds, text, 80, num_beams=3, do_sample=do_sample, top_k=30, top_p=0.8,
                                 seed=7).cpu())
    eng.pl = True
    assert torch.equal(outs[0], outs[1])
