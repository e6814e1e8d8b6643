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


_M64 = (1 << 64) - 1


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _gumbel(key):
    u = (float(_mix64(key & _M64) >> 40) + 0.5) * 5.9604645e-8
    return -np.log(-np.log(u))


@pytest.mark.parametrize("top_k,top_p", [(30, 0.8), (2, 1.0), (64, 0.95), (5, 0.3), (100, 1.0), (0, 0.8),
                                         (200, 0.9)])
def test_beam_candidates_top_k_path_vs_restatement(top_k, top_p):
    """itts_beam_candidates, beam sample with 0 < top_k <= 64 (the reference default top_k 30,
    top_p 0.8 among them), vs a numpy restatement of gpt_beam.hip's contract: log_softmax ->
    repetition penalty -> / T -> TopK (ties at the k-th score kept, <= 64) -> TopP (min 2) ->
    + beam score -> the row's 2K best Gumbel keys (same counter-based noise).  Tokens exact, scores
    and keys to f32 rounding.  Ties are planted at the k-th score."""
    from indextts import _hip
    lib = _hip.load()
    K, B, V = 3, 4, 8194
    R, C = K * B, 2 * K
    ldl = (V + 3) // 4 * 4
    rng = np.random.default_rng(7 + top_k)
    logits = (rng.standard_normal((R, ldl)) * 3).astype(np.float32)
    seen = (rng.random((R, ldl)) < 0.02).astype(np.uint8)
    for r in range(R):  # ties around rank top_k (distinct tokens, equal logits, equal seen flags)
        order = np.argsort(-logits[r, :V], kind="stable")
        logits[r, order[max(top_k - 2, 0): top_k + 2]] = logits[r, order[top_k - 1]]
        seen[r, order[max(top_k - 2, 0): top_k + 2]] = 0
    bscore = (rng.standard_normal(R) * 2).astype(np.float32)
    col, row0, seed = 17, 5, 0x1234_5678_9ABC
    tstate = np.array([col, row0, seed & 0xFFFFFFFF, seed >> 32], dtype=np.int32)
    temp, pen, stop, min_new = 0.9, 1.3, 8193, 0
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    lg, sn, bs, ts = d(logits), d(seen), d(bscore), d(tstate)
    ck = torch.empty(R, C, device="cuda")
    cs = torch.empty(R, C, device="cuda")
    ct = torch.empty(R, C, dtype=torch.int32, device="cuda")
    _hip.check(lib.itts_beam_candidates(lg.data_ptr(), ldl, V, sn.data_ptr(), bs.data_ptr(), ts.data_ptr(), 0, min_new,
                                        stop, pen, 1, temp, top_k, top_p, K, ck.data_ptr(), cs.data_ptr(),
                                        ct.data_ptr(), R, _hip.stream_ptr()), "itts_beam_candidates")
    torch.cuda.synchronize()
    ck, cs, ct = ck.cpu().numpy(), cs.cpu().numpy(), ct.cpu().numpy()
    for r in range(R):
        x = logits[r, :V].astype(np.float64)
        x = x - (x.max() + np.log(np.exp(x - x.max()).sum()))
        x = np.where(seen[r, :V] > 0, np.where(x < 0, x * pen, x / pen), x)
        s = (x / temp).astype(np.float32)
        order = np.lexsort((np.arange(V), -s))
        if 0 < top_k <= 64:  # register path: descending extraction, ties at the k-th kept (<= 64)
            kk = max(top_k, 2)
            tk, tau = [], -np.inf
            for nc, t in enumerate(order[:64]):
                if nc >= kk and s[t] < tau:
                    break
                tk.append(int(t))
                if nc == kk - 1:
                    tau = s[t]
            keep = len(tk)
            if top_p < 1.0 and keep > 2:
                e = np.exp(s[tk].astype(np.float64) - s[tk[0]])
                cum = 0.0
                for i in range(len(tk) - 1, 1, -1):
                    cum += e[i] / e.sum()
                    if cum <= 1.0 - top_p:
                        keep = i
                    else:
                        break
            tk = tk[:keep]
        else:  # general path: HF TopK (k' = max(top_k, 2), ties kept) then HF TopP (min_keep 2)
            keep_m = np.isfinite(s)
            if top_k > 0:
                keep_m &= s >= s[order[max(top_k, 2) - 1]]
            if top_p < 1.0:
                asc = np.argsort(np.where(keep_m, s, -np.inf), kind="stable")
                sv = np.where(keep_m, s, -np.inf)[asc].astype(np.float64)
                pr = np.exp(sv - sv.max())
                cum = np.cumsum(pr / pr.sum())
                rem = cum <= 1.0 - top_p
                rem[-2:] = False
                keep_m[asc[rem]] = False
            tk = [int(t) for t in order if keep_m[t]]
        rkey = _mix64(seed ^ _mix64((((r + row0) & 0xFFFFFFFF) << 32) | col))
        score = np.array([s[t] + bscore[r] for t in tk])
        key = np.array([score[i] + _gumbel(rkey + t + 1) for i, t in enumerate(tk)])
        best = np.lexsort((np.array(tk), -key))[:C]
        n = len(best)
        assert ct[r].tolist() == [tk[i] for i in best] + [stop] * (C - n), (r, ct[r], [tk[i] for i in best])
        np.testing.assert_allclose(cs[r, :n], score[best], rtol=0, atol=2e-4)
        np.testing.assert_allclose(ck[r, :n], key[best], rtol=0, atol=2e-3)
        assert np.all(np.isneginf(ck[r, n:])) and np.all(np.isneginf(cs[r, n:]))


@pytest.mark.parametrize("K", [5, 12, 16])
def test_f32_wide_beam_search_matches_oracle(beam_golden, K):
    """num_beams up to 16 (candidate tables of 16 x 32 in LDS, 8 per lane in the per-utterance merge):
    f32 beam search ids equal the oracle's HF 4.36 beam_search restatement (pinned to the reference's
    own num_beams = 2, 3 goldens, tests/test_oracle_beam.py) on the tiny config, single and padded
    batch, with the stop logit raised so hypotheses close mid-run."""
    from oracle.gpt_oracle import GPTOracle
    bg = beam_golden
    sd = _sd("tiny", 5.0, bg)
    eng = _engine("tiny", "f32", 5.0, bg)
    o = GPTOracle({k: v.clone() for k, v in sd.items()}, _cfg("tiny").gpt)
    n = int(bg["tiny_steps"])
    conds = torch.from_numpy(bg["tiny_conds"])
    for text in (torch.from_numpy(bg["tiny_text"]), torch.from_numpy(bg["tiny_batch_text"])):
        want = o.generate_beam(conds, text, n, num_beams=K).numpy()
        got = eng.generate(conds.cuda(), text.cuda(), n, num_beams=K, check_every=1).cpu().numpy()
        np.testing.assert_array_equal(got, want)
