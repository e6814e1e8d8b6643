"""bf16 product-path parity of the decoding srt_dubbing actually runs, and a tighter greedy leg
(VERDICT r05, next 1).

srt_dubbing filters its kwargs through ``inspect.signature(infer)``, so every cue decodes with the
reference defaults: beam sample, ``num_beams=3`` (reference ``infer.py:535-543`` ->
``gpt/model.py:655-708``, transformers 4.36 ``beam_sample``).  The tests here pin the FULL-SIZE bf16
product path (IndexTTS-1.5 shape, MFMA decode, persistent layers / launch chain) against the CPU oracle
(``oracle/gpt_oracle.py``, pinned to the reference's own goldens by ``tests/test_oracle_*.py``):

  * beam search (``do_sample=False``), 32 steps, EOS held off (``min_new_tokens``): at 32 utterances
    (96 beam rows, the persistent layers) and at 128 utterances (384 rows, srt_dubbing's chunk: the launch
    chain).  Every step's beam SET per utterance (sequences; scores within the measured error) equals the
    oracle's, at every step before the utterance's first candidate near-tie -- the oracle's K-th vs K+1-th
    candidate gap <= 2x a candidate's measured error bound (its parent beam's score error at the step before +
    the largest one-step log-prob error measured).  Checked against the oracle on the bf16 weights the GPU
    stores (activation rounding is the only difference left) and on the fp32 master weights.
  * beam sample (``do_sample=True``, top_k 30, top_p 0.8, the reference defaults) at full size on the
    persistent layers: the distributions of the first two output tokens equal the oracle's -- a two-sample
    permutation test on the total-variation distance (p > 0.002).
  * greedy against the oracle run on the bf16-ROUNDED weights (``parity_util.bf16_effective_gpt_sds``):
    the remaining logit error is activation rounding only, so the bars are tighter than the fp32 leg's
    (``test_gpu_fullsize.py``), and free-running agreement must hold up to the oracle's first near-tie.
Measured values go to the parity record (``parity_util.record``).
"""
import os

import numpy as np
import pytest
import torch

from parity_util import bf16_effective_gpt_sds, record

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
# bf16 decode vs the oracle on the bf16-rounded weights: raw-logit bar (<= 1.5x the measured value,
# profiles/parity_r06*.json)
LOGIT_ERR_W = 0.041  # measured 0.0275 (profiles/parity_r06a.json)
_cache = {}


def _cfg():
    from indextts.utils.config import default_config_path, load_config
    return load_config(default_config_path())


def _sd(head_std=0.08):
    key = ("sd", head_std)
    if key not in _cache:
        from indextts.utils.synthetic import gpt_state_dict
        _cache[key] = {k: torch.from_numpy(np.asarray(v)).clone()
                       for k, v in gpt_state_dict(_cfg().gpt, 0, head_std).items()}
    return _cache[key]


def _engine(max_kv, head_std=0.08):
    key = ("eng", max_kv, head_std)
    if key not in _cache:
        from indextts.gpt.engine import HipGPT
        for k in [k for k in _cache if k[0] == "eng"]:
            del _cache[k]
        torch.cuda.empty_cache()
        _cache[key] = HipGPT(_sd(head_std), _cfg().gpt, "cuda", dtype="bf16", max_kv=max_kv)
    return _cache[key]


def _oracle(kind, head_std=0.08):
    """kind "fp32": the master weights; "bf16w": the weights as the bf16 product path stores them."""
    key = ("orc", kind, head_std)
    if key not in _cache:
        from oracle.gpt_oracle import GPTOracle
        cfg = _cfg()
        if kind == "fp32":
            _cache[key] = GPTOracle(_sd(head_std), cfg.gpt)
        else:
            pre, dec = bf16_effective_gpt_sds(_sd(head_std), int(cfg.gpt.layers))
            _cache[key] = GPTOracle(pre, cfg.gpt, sd_decode=dec)
    return _cache[key]


# ------------------------------------------------------------------------------------------- greedy
@pytest.fixture(scope="module")
def c2():
    return np.load(os.path.join(HERE, "golden", "golden_c2.npz"))


def _processed(logits, fed, penalty=10.0):
    """[n, V] raw logits of n steps fed ``fed`` [n] -> the scores greedy picks from (repetition penalty over
    the fake prefix ids and every earlier code; EOS excluded: the steps run under min_new_tokens)."""
    n, V = logits.shape
    seen = torch.zeros(n, V, dtype=torch.bool)
    seen[:, 1] = seen[:, 8192] = True
    f = torch.zeros(n, V, dtype=torch.int32)
    f[torch.arange(1, n), fed[: n - 1].long()] = 1
    seen |= f.cumsum(0) > 0
    sc = torch.where(seen, torch.where(logits < 0, logits * penalty, logits / penalty), logits)
    sc[:, 8193] = float("-inf")
    return sc


def test_c2_bf16_vs_bf16_weight_oracle(c2):
    """C2 (B = 1, L = 48, 511-frame prompt, 400 EOS-suppressed steps, keys 83 -> 483).
    (1) teacher-forced on the reference's ids: raw logits within LOGIT_ERR_W of the bf16-weight oracle's;
    ids equal wherever the oracle's top-1 / top-2 margin exceeds 2x the measured processed-score error.
    (2) free-running: the GPU's ids equal the bf16-weight oracle's free-running ids at every step before the
    oracle's first near-tie (margin <= 2x that error); the agreement length is recorded."""
    eng = _engine(576)
    orc = _oracle("bf16w")
    conds, text = torch.from_numpy(c2["c2_conds"]), torch.from_numpy(c2["c2_text"])
    ref = torch.from_numpy(c2["c2_codes"])
    n = ref.shape[1]
    eng.logits_trace = []
    try:
        got = eng.generate(conds.cuda(), text.cuda(), n, min_new_tokens=n, forced_codes=ref.cuda()).cpu()[0]
        gl = torch.cat(eng.logits_trace, 0).cpu()
    finally:
        eng.logits_trace = None
    with torch.no_grad():
        ol = orc.forced_logits(conds, text, ref)[0]
        olf = _oracle("fp32").forced_logits(conds, text, ref)[0]
    raw = float((gl - ol).abs().max())
    raw_fp32 = float((gl - olf).abs().max())
    wround = float((ol - olf).abs().max())  # what the weight rounding alone moves the oracle's logits
    gp, op = _processed(gl, ref[0]), _processed(ol, ref[0])
    top2 = torch.topk(op, 2, dim=1)
    comp = op >= top2.values[:, :1] - 1.0
    err = float((gp - op).abs()[comp].max())
    marg = (top2.values[:, 0] - top2.values[:, 1]).numpy()
    sure = marg > max(2 * err, 1e-3)
    bad = np.nonzero((got.numpy() != top2.indices[:, 0].numpy()) & sure)[0]
    print(f"c2 bf16 vs bf16-weight oracle, {n} forced steps: raw |err| {raw:.4f} (vs fp32 oracle {raw_fp32:.4f}; "
          f"weight rounding alone moves the oracle {wround:.4f}); processed {err:.4f}; "
          f"{int((~sure).sum())} steps under 2x err")
    # (2) free running, both sides
    eng.logits_trace = []
    try:
        free = eng.generate(conds.cuda(), text.cuda(), n, min_new_tokens=n).cpu()[0].numpy()
        fl = torch.cat(eng.logits_trace, 0).cpu()
    finally:
        eng.logits_trace = None
    with torch.no_grad():
        ofree, otr = orc.generate(conds, text, n, min_new_tokens=n, return_trace=True)
    ofree = ofree[0].numpy()
    omarg = np.array([float(m[0]) for _, m in otr])
    diff = np.nonzero(free != ofree)[0]
    agree = int(diff[0]) if diff.size else n
    m_err = err
    if agree > 0:  # the free-running processed-score error on the common prefix
        fp, fo = _processed(fl[:agree], torch.from_numpy(ofree)), torch.stack([t[0][0] for t in otr[:agree]])
        fo = fo.clone()
        fo[:, 8193] = float("-inf")
        cmp = fo >= fo.max(dim=1, keepdim=True).values - 1.0
        m_err = max(err, float((fp - fo).abs()[cmp].max()))
    ties = np.nonzero(omarg <= max(2 * m_err, 1e-3))[0]
    first_tie = int(ties[0]) if ties.size else n
    print(f"c2 free running: ids agree with the bf16-weight oracle for {agree} of {n} steps; the oracle's first "
          f"near-tie (margin <= {2 * m_err:.4f}) at step {first_tie}")
    record("c2_bf16_vs_bf16w_oracle", raw_logit_err=raw, raw_logit_err_fp32_oracle=raw_fp32,
           weight_rounding_logit_shift=wround, score_err=err, exempt_steps=int((~sure).sum()), steps=n,
           exempt_id_diffs=int(((got.numpy() != top2.indices[:, 0].numpy()) & ~sure).sum()),
           free_running_agree=agree, free_running_first_tie=first_tie, free_running_score_err=m_err, bound=LOGIT_ERR_W)
    assert bad.size == 0, (bad[:10], marg[bad[:10]])
    assert raw <= LOGIT_ERR_W and err <= LOGIT_ERR_W, (raw, err)
    assert agree >= first_tie, (agree, first_tie)


# ------------------------------------------------------------------------------------ beam search
def _beam_inputs(B, seed):
    g = torch.Generator().manual_seed(seed)
    lens = [int(torch.randint(12, 25, (1,), generator=g)) for _ in range(B)]
    L = max(lens)
    text = torch.stack([torch.nn.functional.pad(torch.randint(2, 12000, (n,), generator=g), (0, L - n), value=1)
                        for n in lens])
    conds = torch.randn(B, 32, 1024, generator=g)
    return conds, text


def _beam_sets(codes, scores, b, K):
    """utterance b's beams as {sequence: score}"""
    return {tuple(codes[b * K + k].tolist()): float(scores[b * K + k]) for k in range(K)}


def _compare_beams(gtr, otr, U, K):
    """GPU trace (codes [R, t+1], scores [R], done [B]) vs oracle trace (seqs, scores [B', K], vals [B', 2K]) per
    step, for GPU utterances U[u] = oracle utterance u -> dict of
      first_bad [U]: the first step whose beam set differs;
      E [n, U]: max |GPU - oracle| beam score at each step while the sets are equal (NaN after);
      e1: max |error| of one step's score increment (a beam's score minus its parent's: the step's processed
          log-prob), over every matched beam -- what a single step adds to a candidate's error;
      gaps [n, U]: the oracle's K-th vs K+1-th candidate gap of each step."""
    n = min(len(gtr), len(otr))
    first_bad = np.full(len(U), n)
    E = np.full((n, len(U)), np.nan)
    gaps = np.zeros((n, len(U)))
    e1 = 0.0
    prev = [None] * len(U)
    for t in range(n):
        gc, gs, _ = gtr[t]
        oe = otr[t]
        for u, b in enumerate(U):
            gaps[t, u] = float(oe["vals"][u, K - 1] - oe["vals"][u, K])
            if first_bad[u] < n:
                continue
            gset = _beam_sets(gc, gs, b, K)
            oset = {tuple(oe["seqs"][u * K + k]): float(oe["scores"][u, k]) for k in range(K)}
            if set(gset) != set(oset):
                first_bad[u] = t
                continue
            E[t, u] = max(abs(gset[q] - oset[q]) for q in gset)
            for q in gset:  # the step's increment vs the parent's (t = 0: the parent is the empty prefix)
                gp, op = (0.0, 0.0) if t == 0 else prev[u][q[:-1]]
                e1 = max(e1, abs((gset[q] - gp) - (oset[q] - op)))
            prev[u] = {q: (gset[q], oset[q]) for q in gset}
    return {"first_bad": first_bad, "E": E, "e1": e1, "gaps": gaps}


@pytest.mark.parametrize("B,U,path", [(32, tuple(range(32)), "pl"), (128, tuple(range(0, 128, 8)), "chain")])
def test_bf16_beam_search_sets_equal_oracle(B, U, path):
    """bf16 beam search (num_beams 3, do_sample False, the reference's repetition penalty 10), 32 steps, EOS
    held off: at B = 32 (96 rows) on the persistent layers, at B = 128 (384 rows, srt_dubbing's chunk) on the
    launch chain.  For the utterances U, every step's beam set equals the oracle's (bf16-weight oracle, and the
    fp32 one on the first 8) until the utterance's first candidate near-tie: the oracle's K-th vs K+1-th
    candidate gap <= 2x the measured beam-score error."""
    K, n = 3, 32
    conds, text = _beam_inputs(B, 600 + B)
    eng = _engine(32 + text.shape[1] + 2 + 1 + n + 8)
    assert eng.pl_takes(B * K, beams=True) == (path == "pl"), "the shape runs on the intended decode path"
    eng.beam_trace = []
    try:
        out = eng.generate(conds.cuda(), text.cuda(), n, num_beams=K, min_new_tokens=n).cpu().numpy()
        gtr = eng.beam_trace
        ran_pl = eng._pl_ran
    finally:
        eng.beam_trace = None
    assert ran_pl == (path == "pl")
    assert len(gtr) == n
    for kind, sub in (("bf16w", list(U)), ("fp32", list(U)[:8])):
        otr = []
        with torch.no_grad():
            want = _oracle(kind).generate_beam(conds[sub], text[sub], n, num_beams=K, min_new_tokens=n, trace=otr)
        cmp = _compare_beams(gtr, otr, sub, K)
        first_bad, E, e1, gaps = cmp["first_bad"], cmp["E"], cmp["e1"], cmp["gaps"]
        # a candidate at step t = a beam of step t-1 (error <= E[t-1]) + one step's log-prob (error <= e1): the
        # selection is determined unless the oracle's K-th / K+1-th gap is within twice that
        err_prev = np.vstack([np.zeros((1, len(sub))), np.nan_to_num(E[:-1], nan=np.inf)])
        ties = gaps <= 2 * (err_prev + e1)
        first_tie = np.where(ties.any(0), ties.argmax(0), n)
        full = first_bad >= n
        same_out = [bool(np.array_equal(out[b, : want.shape[1]], want[u].numpy())) for u, b in enumerate(sub)]
        err = float(np.nanmax(E))
        print(f"beam3 B={B} ({path}) vs {kind} oracle on {len(sub)} utterances: beam-score err max {err:.4f}, "
              f"one step's log-prob err {e1:.4f}; first near-tie step min {first_tie.min()} / median "
              f"{float(np.median(first_tie))} of {n}; beam sets equal at every step in {int(full.sum())} of {len(sub)} "
              f"(first difference: median {float(np.median(first_bad))}); equal through the first near-tie in "
              f"{int((first_bad >= first_tie).sum())} of {len(sub)}; identical outputs: {sum(same_out)} "
              f"(all {int(full.sum())} with equal sets: {all(s for s, f in zip(same_out, full) if f)})")
        record(f"beam3_b{B}_{path}_vs_{kind}", score_err=err, step_logprob_err=e1, utterances=len(sub), steps=n,
               first_tie_min=int(first_tie.min()), first_tie_median=float(np.median(first_tie)),
               first_mismatch_min=int(first_bad.min()), first_mismatch_median=float(np.median(first_bad)),
               agree_all_steps=int(full.sum()), identical_outputs=int(sum(same_out)))
        assert (first_bad >= first_tie).all(), (kind, first_bad, first_tie)
        assert all(s for s, f in zip(same_out, full) if f), (kind, same_out)
        assert e1 <= LOGIT_ERR_W * 2 and err <= 0.15, (e1, err)  # measured 0.066-0.068 (32 steps)


# ------------------------------------------------------------------------------------ beam sample
def _tv_test(a, b, n_perm=2000, seed=0):
    """two-sample permutation test of total-variation distance -> (tv, p-value)"""
    def tv(x, y):
        k = int(max(x.max(), y.max())) + 1
        return 0.5 * np.abs(np.bincount(x, minlength=k) / len(x) - np.bincount(y, minlength=k) / len(y)).sum()
    obs = tv(a, b)
    pool = np.concatenate([a, b])
    rng = np.random.default_rng(seed)
    hits = 0
    for _ in range(n_perm):
        rng.shuffle(pool)
        hits += tv(pool[: len(a)], pool[len(a):]) >= obs - 1e-12
    return obs, (hits + 1) / (n_perm + 1)


def test_bf16_beam_sample_distribution_full_size_on_persistent_layers():
    """the reference default decoding (num_beams 3, do_sample, top_k 30, top_p 0.8, T 1), full size, bf16,
    32 utterances per call (96 rows: the persistent layers), 20 calls with distinct seeds = 640 draws, against
    400 draws of the fp32 oracle's HF 4.36 beam_sample restatement: the first and the second output token's
    distributions agree (permutation test on the total-variation distance, p > 0.002 each)."""
    K, n, N, calls = 3, 3, 32, 20
    conds, text = _beam_inputs(1, 77)
    eng = _engine(32 + text.shape[1] + 2 + 1 + n + 8)
    assert eng.pl_takes(N * K, beams=True)
    got = []
    for i in range(calls):
        out = eng.generate(conds.cuda().expand(N, -1, -1).contiguous(), text.cuda().expand(N, -1).contiguous(), n,
                           num_beams=K, do_sample=True, top_k=30, top_p=0.8, seed=1000 + i)
        assert eng._pl_ran
        got.append(out[:, :2].cpu().numpy())
    got = np.concatenate(got, 0)
    gen = torch.Generator().manual_seed(0)
    with torch.no_grad():
        ref = _oracle("fp32").generate_beam(conds, text, n, num_beams=K, do_sample=True, top_k=30, top_p=0.8,
                                            generator=gen, copies=400).numpy()
    res = {}
    for j in range(2):
        tv, p = _tv_test(got[:, j], ref[:, j], seed=j)
        res[j] = (tv, p)
        print(f"beam sample token {j}: TV {tv:.3f} (p = {p:.3f}); GPU top {np.bincount(got[:, j]).argsort()[-3:][::-1]}, "
              f"oracle top {np.bincount(ref[:, j]).argsort()[-3:][::-1]}")
    record("beam_sample_full_bf16_pl", tv_token0=res[0][0], p_token0=res[0][1], tv_token1=res[1][0],
           p_token1=res[1][1], gpu_draws=len(got), oracle_draws=len(ref))
    assert res[0][1] > 0.002 and res[1][1] > 0.002, res
