"""GPU beam search / beam sample (gpt_beam.hip + itts_attn_decode_rows) through the C ABI.

Contract:
  * beam search (do_sample=False), f32 verification mode: ids bit-exact vs the REFERENCE's
    inference_speech(num_beams=K) goldens (tests/golden/beam_golden.npz, K = 2, 3; single, padded
    batch, min_new_tokens, stop logit raised so hypotheses close mid-run / early stop fires), with and
    without the hipGraph;
  * bf16 product mode: batch-invariant ids (an utterance decodes identically alone and inside a
    batch of 32: the kernels are row/utterance independent) and the first ids equal the reference's;
  * beam sample: the oracle's restatement and the GPU agree in distribution (first-token frequencies).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

_cache = {}


def _cfg(tag):
    from indextts.utils.config import default_config_path, load_config, tiny_config
    return tiny_config() if tag == "tiny" else load_config(default_config_path())


def _sd(tag, boost, bg):
    from indextts.utils.synthetic import gpt_state_dict
    cfg = _cfg(tag)
    sd = {k: torch.from_numpy(np.asarray(v)).clone()
          for k, v in gpt_state_dict(cfg.gpt, 0, float(bg[f"{tag}_head_std"])).items()}
    sd["mel_head.bias"][int(cfg.gpt.stop_mel_token)] += boost
    return sd


def _engine(tag, mode, boost, bg, max_kv=256):
    key = (tag, mode, boost, max_kv)
    if key not in _cache:
        from indextts.gpt.engine import HipGPT
        _cache.clear()
        torch.cuda.empty_cache()
        _cache[key] = HipGPT(_sd(tag, boost, bg), _cfg(tag).gpt, "cuda", dtype=mode, max_kv=max_kv)
    return _cache[key]


@pytest.mark.parametrize("tag", ["tiny", "full"])
@pytest.mark.parametrize("graph", [True, False])
def test_f32_beam_search_ids_bit_exact(beam_golden, tag, graph):
    bg = beam_golden
    eng = _engine(tag, "f32", 0.0, bg)
    conds = torch.from_numpy(bg[f"{tag}_conds"]).cuda()
    text = torch.from_numpy(bg[f"{tag}_text"]).cuda()
    n = int(bg[f"{tag}_steps"])
    got = eng.generate(conds, text, n, num_beams=3, use_graph=graph).cpu().numpy()
    np.testing.assert_array_equal(got, bg[f"{tag}_codes"])
    got = eng.generate(conds, text, n, num_beams=2, use_graph=graph).cpu().numpy()
    np.testing.assert_array_equal(got, bg[f"{tag}_codes_k2"])
    got = eng.generate(conds, text, n, num_beams=3, min_new_tokens=n // 2, use_graph=graph).cpu().numpy()
    np.testing.assert_array_equal(got, bg[f"{tag}_codes_minnew"])
    batch = torch.from_numpy(bg[f"{tag}_batch_text"]).cuda()
    got = eng.generate(conds, batch, n, num_beams=3, use_graph=graph).cpu().numpy()
    np.testing.assert_array_equal(got, bg[f"{tag}_codes_batch"])


@pytest.mark.parametrize("tag,boost", [("tiny", 5.0), ("tiny", 6.0), ("full", 4.0), ("full", 6.0)])
def test_f32_beam_search_eos_hypotheses_bit_exact(beam_golden, tag, boost):
    bg = beam_golden
    eng = _engine(tag, "f32", boost, bg)
    conds = torch.from_numpy(bg[f"{tag}_conds"]).cuda()
    batch = torch.from_numpy(bg[f"{tag}_batch_text"]).cuda()
    got = eng.generate(conds, batch, int(bg[f"{tag}_steps"]), num_beams=3, check_every=1).cpu().numpy()
    np.testing.assert_array_equal(got, bg[f"{tag}_eos{boost:g}_codes_batch"])


def test_bf16_beam_search_batch_invariant_and_close(beam_golden):
    bg = beam_golden
    eng = _engine("full", "bf16", 0.0, bg, max_kv=32 + 14 + 2 + 1 + 64 + 8)
    conds = torch.from_numpy(bg["full_conds"]).cuda()
    text = torch.from_numpy(bg["full_text"]).cuda()
    n = int(bg["full_steps"])
    alone = eng.generate(conds, text, n, num_beams=3).cpu().numpy()
    g = torch.Generator().manual_seed(5)
    others = torch.randint(2, 12000, (31, text.shape[1]), generator=g).cuda()
    batch = torch.cat([others[:13], text, others[13:]], 0)
    many = eng.generate(conds, batch, n, num_beams=3).cpu().numpy()
    np.testing.assert_array_equal(many[13, : alone.shape[1]], alone[0])
    assert (many[13, alone.shape[1]:] == 8193).all()
    np.testing.assert_array_equal(alone[0, :4], bg["full_codes"][0, :4])


@pytest.mark.parametrize("top_k,top_p", [(30, 0.8), (0, 0.8), (100, 1.0)])
def test_beam_sample_distribution_matches_oracle(beam_golden, top_k, top_p):
    """tiny config, reference defaults (top_k 30, top_p 0.8, T 1, 3 beams) and the general warper
    path (top-p only; top_k > 64), 3 steps: total-variation distance between the GPU's and the
    oracle's first-token distributions <= 0.12 (600 GPU samples in one batched call vs 400 oracle
    samples)."""
    from oracle.gpt_oracle import GPTOracle
    bg = beam_golden
    eng = _engine("tiny", "f32", 0.0, bg)
    conds = torch.from_numpy(bg["tiny_conds"])
    text = torch.from_numpy(bg["tiny_text"])
    N = 600
    got = eng.generate(conds.cuda(), text.cuda().expand(N, -1).contiguous(), 3, num_beams=3, do_sample=True,
                       top_k=top_k, top_p=top_p, seed=123).cpu().numpy()
    orc = GPTOracle(_sd("tiny", 0.0, bg), _cfg("tiny").gpt)
    gen = torch.Generator().manual_seed(0)
    ref = [int(orc.generate_beam(conds, text, 3, do_sample=True, top_k=top_k, top_p=top_p, generator=gen)[0, 0])
           for _ in range(400)]
    pg = np.bincount(got[:, 0], minlength=8194) / N
    pr = np.bincount(np.array(ref), minlength=8194) / len(ref)
    tv = 0.5 * np.abs(pg - pr).sum()
    assert tv <= 0.12, (tv, np.argsort(-pg)[:5], np.sort(-pg)[:5], np.argsort(-pr)[:5], np.sort(-pr)[:5])
    # different seeds -> different draws; same seed -> same draws
    again = eng.generate(conds.cuda(), text.cuda().expand(N, -1).contiguous(), 3, num_beams=3, do_sample=True,
                         top_k=top_k, top_p=top_p, seed=123).cpu().numpy()
    np.testing.assert_array_equal(again, got)
