"""Pin the oracle's beam-search restatement (HF 4.36 beam_search / beam_sample + BeamSearchScorer,
oracle/gpt_oracle.py ``generate_beam``) against the REFERENCE's ``inference_speech(num_beams=K)``
(tests/golden/make_beam_golden.py).  CPU only.  Bar: bit-exact ids."""
import numpy as np
import pytest
import torch

from indextts.utils.config import default_config_path, load_config, tiny_config
from indextts.utils.synthetic import gpt_state_dict
from oracle.gpt_oracle import GPTOracle

_cache = {}


def oracle(tag, boost, bg):
    key = (tag, boost)
    if key not in _cache:
        cfg = tiny_config() if tag == "tiny" else load_config(default_config_path())
        sd = {k: torch.from_numpy(np.asarray(v)).clone()
              for k, v in gpt_state_dict(cfg.gpt, 0, float(bg[f"{tag}_head_std"])).items()}
        sd["mel_head.bias"][int(cfg.gpt.stop_mel_token)] += boost
        _cache[key] = GPTOracle(sd, cfg.gpt)
    return _cache[key]


@pytest.mark.parametrize("tag", ["tiny", "full"])
def test_beam_search_ids_match_reference(beam_golden, tag):
    bg = beam_golden
    o = oracle(tag, 0.0, bg)
    conds, text, n = torch.from_numpy(bg[f"{tag}_conds"]), torch.from_numpy(bg[f"{tag}_text"]), int(bg[f"{tag}_steps"])
    with torch.no_grad():
        np.testing.assert_array_equal(o.generate_beam(conds, text, n).numpy(), bg[f"{tag}_codes"])
        np.testing.assert_array_equal(o.generate_beam(conds, text, n, num_beams=2).numpy(), bg[f"{tag}_codes_k2"])
        np.testing.assert_array_equal(o.generate_beam(conds, text, n, min_new_tokens=n // 2).numpy(),
                                      bg[f"{tag}_codes_minnew"])
        batch = torch.from_numpy(bg[f"{tag}_batch_text"])
        np.testing.assert_array_equal(o.generate_beam(conds, batch, n).numpy(), bg[f"{tag}_codes_batch"])


@pytest.mark.parametrize("tag,boost", [("tiny", 5.0), ("tiny", 6.0), ("full", 4.0), ("full", 6.0)])
def test_beam_search_eos_hypotheses_match_reference(beam_golden, tag, boost):
    """stop logit raised: hypotheses close mid-run, utterances finish at different steps."""
    bg = beam_golden
    o = oracle(tag, boost, bg)
    conds, n = torch.from_numpy(bg[f"{tag}_conds"]), int(bg[f"{tag}_steps"])
    with torch.no_grad():
        got = o.generate_beam(conds, torch.from_numpy(bg[f"{tag}_batch_text"]), n)
    np.testing.assert_array_equal(got.numpy(), bg[f"{tag}_eos{boost:g}_codes_batch"])


def test_warpers_match_hf_definitions():
    """top-k keeps ties at the k-th value and at least min_keep; top-p drops the low tail whose
    cumulative probability <= 1 - p, keeping at least min_keep."""
    sc = torch.tensor([[0.0, -1.0, -1.0, -3.0, -5.0, -0.5]])
    out = GPTOracle.warp(sc, 1.0, 2, 1.0, 2)
    assert torch.isfinite(out).tolist() == [[True, False, False, False, False, True]]
    out = GPTOracle.warp(sc, 1.0, 3, 1.0, 2)  # tie at the 3rd value: both kept
    assert torch.isfinite(out).sum() == 4
    p = torch.log(torch.tensor([[0.5, 0.3, 0.15, 0.05]]))
    out = GPTOracle.warp(p, 1.0, 0, 0.8, 1)
    assert torch.isfinite(out).tolist() == [[True, True, False, False]]
    out = GPTOracle.warp(p, 1.0, 0, 0.1, 2)  # min_keep 2
    assert torch.isfinite(out).sum() == 2


def test_beam_sample_first_token_distribution(beam_golden):
    """beam_sample, 1 step: every beam starts at score 0 and the first-step rows are identical, so each
    of the 2K draws is a draw without replacement from K copies of the warped distribution; the
    best-scored non-eos draw is the first token of the returned sequence.  Its empirical distribution
    must match the analytic one (top token of K x top-k candidates)."""
    bg = beam_golden
    o = oracle("tiny", 0.0, bg)
    conds, text = torch.from_numpy(bg["tiny_conds"]), torch.from_numpy(bg["tiny_text"])
    g = torch.Generator().manual_seed(0)
    counts = {}
    with torch.no_grad():
        for _ in range(300):
            t = int(o.generate_beam(conds, text, 1, do_sample=True, top_k=3, top_p=1.0, generator=g)[0, 0])
            counts[t] = counts.get(t, 0) + 1
    assert len(counts) <= 3  # only the top-3 tokens survive the warper
    assert max(counts.values()) > 100  # the most likely token wins most often


def test_oracle_test_conveniences_keep_semantics(beam_golden):
    """``copies`` / ``trace`` of generate_beam and the split prefill / decode weights (``sd_decode``) are
    test conveniences: copies decode like the utterance repeated, the trace's last entry is the returned
    state, and ``sd_decode`` = the same weights changes nothing (tiny config, CPU)."""
    bg = beam_golden
    o = oracle("tiny", 0.0, bg)
    conds, text, n = torch.from_numpy(bg["tiny_conds"]), torch.from_numpy(bg["tiny_text"]), 12
    with torch.no_grad():
        one = o.generate_beam(conds, text, n)
        tr = []
        rep = o.generate_beam(conds, text, n, copies=3, trace=tr)
        assert torch.equal(rep, one.expand(3, -1))
        assert len(tr) == n and len(tr[-1]["seqs"]) == 9 and tr[-1]["vals"].shape == (3, 6)
        assert all(len(q) == n for q in tr[-1]["seqs"])
        o2 = GPTOracle({k: v.clone() for k, v in o.sd.items()}, tiny_config().gpt, sd_decode=o.sd)
        assert torch.equal(o2.generate_beam(conds, text, n), one)
        assert torch.equal(o2.generate(conds, text, n), o.generate(conds, text, n))
        codes = o.generate(conds, text, n)
        np.testing.assert_allclose(o2.forced_logits(conds, text, codes).numpy(),
                                   o.forced_logits(conds, text, codes).numpy(), rtol=0, atol=2e-4)


def test_bf16_effective_fold_is_exact_without_rounding():
    """tests/parity_util.bf16_effective_gpt_sds (the bf16 product path's weight forms for the oracle): with the
    rounding off, folding ln_1 / ln_2 into c_attn / c_fc is the same function (logits within f32 noise), and
    with it on the logits move by a small amount (the weight rounding the GPU leg isolates)."""
    from parity_util import bf16_effective_gpt_sds
    cfg = tiny_config()
    sd = {k: torch.from_numpy(np.asarray(v)).clone() for k, v in gpt_state_dict(cfg.gpt, 3, 0.15).items()}
    g = torch.Generator().manual_seed(1)
    for i in range(int(cfg.gpt.layers)):  # non-trivial LayerNorm affines
        for ln in ("ln_1", "ln_2"):
            sd[f"gpt.h.{i}.{ln}.weight"] = 1 + 0.2 * torch.randn(sd[f"gpt.h.{i}.{ln}.weight"].shape, generator=g)
            sd[f"gpt.h.{i}.{ln}.bias"] = 0.1 * torch.randn(sd[f"gpt.h.{i}.{ln}.bias"].shape, generator=g)
    conds = torch.randn(1, 32, int(cfg.gpt.model_dim), generator=g)
    text = torch.randint(2, 200, (1, 10), generator=g)
    base = GPTOracle(sd, cfg.gpt)
    with torch.no_grad():
        codes = base.generate(conds, text, 16, min_new_tokens=16)
        want = base.forced_logits(conds, text, codes)
        pre, dec = bf16_effective_gpt_sds(sd, int(cfg.gpt.layers), rounding=False)
        exact = GPTOracle(pre, cfg.gpt, sd_decode=dec).forced_logits(conds, text, codes)
        pre, dec = bf16_effective_gpt_sds(sd, int(cfg.gpt.layers))
        rounded = GPTOracle(pre, cfg.gpt, sd_decode=dec).forced_logits(conds, text, codes)
    assert float((exact - want).abs().max()) < 1e-4
    d = float((rounded - want).abs().max())
    assert 1e-4 < d < 0.2, d
