"""Batched pipeline determinism and the pipelined multi-batch driver (BatchedTTS.synthesize_many):
two identical calls give identical PCM (MIOpen asked for deterministic convs in conditioning /
ECAPA), and the two-stream pipelined driver returns exactly what ``synthesize`` returns per batch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tts():
    from indextts.pipeline import BatchedTTS
    from indextts.utils.config import tiny_config
    from indextts.utils.synthetic import bigvgan_state_dict, gpt_state_dict
    cfg = tiny_config()
    return BatchedTTS(gpt_state_dict(cfg.gpt, 0, mel_head_std=0.15), bigvgan_state_dict(cfg.bigvgan, 0), cfg, "cuda",
                      "bf16", max_kv=256)


def _inputs(cfg, n, seed):
    g = np.random.default_rng(seed)
    mels = [torch.from_numpy(g.normal(-4, 2, (1, 100, int(g.integers(60, 90)))).astype(np.float32)).cuda()
            for _ in range(n)]
    texts = [torch.from_numpy(g.integers(2, int(cfg.gpt.number_text_tokens), int(g.integers(6, 14)))).cuda()
             for _ in range(n)]
    return mels, texts


def _same(a, b):
    n = a[1]
    assert torch.equal(a[1], b[1])
    assert all(torch.equal(x, y) for x, y in zip(a[2], b[2]))
    for i in range(len(n)):
        assert torch.equal(a[0][i, : int(n[i])], b[0][i, : int(n[i])]), i


def test_synthesize_is_deterministic(tts):
    mels, texts = _inputs(tts.cfg, 6, 1)
    r1 = tts.synthesize(mels, texts, max_mel_tokens=24)
    r2 = tts.synthesize(mels, texts, max_mel_tokens=24)
    torch.cuda.synchronize()
    _same(r1, r2)


@pytest.mark.parametrize("overlap", [None, True, False])
def test_synthesize_many_equals_synthesize(tts, overlap):
    """auto (5-row batches: every decode fits the persistent layers -> back to back on one stream), forced
    overlap (decode on the launch chain beside the back stream) and forced serial: all equal synthesize"""
    batches = [_inputs(tts.cfg, 5, s) for s in (2, 3, 4)]
    want = [tts.synthesize(m, t, max_mel_tokens=24) for m, t in batches]
    got = tts.synthesize_many(batches, max_mel_tokens=24, overlap=overlap)
    torch.cuda.synchronize()
    for w, g in zip(want, got):
        _same(w, g)
