"""A CPU stand-in for ``indextts.infer.IndexTTS`` (no GPU): the real lookahead / device-pool control
logic of IndexTTS with a deterministic fake synthesis underneath (PCM = a function of the text and
the decoding arguments), for the CPU tests of cross-call batching and of the worker protocol."""
import zlib

import numpy as np

from indextts.infer import IndexTTS

POISON = "this cue makes synthesis fail"


def fake_pcm(text, gen):
    seed = zlib.crc32(repr((text, sorted(gen.items()))).encode())
    n = 3 + len(text) % 7
    return np.random.default_rng(seed).integers(-30000, 30000, (n, 1)).astype(np.int16)


class _Tok:
    def tokenize(self, text):
        return text.split()


class StubTTS(IndexTTS):
    """IndexTTS whose synthesis is fake; ``calls`` records every batched / single synthesis."""

    def __init__(self, cfg_path=None, model_dir=None, is_fp16=True, device="cuda:0", use_cuda_kernel=None, pool=None):
        self.device = str(device)
        self._pool = pool
        self.tokenizer = _Tok()
        self.calls = []

    def infer_many(self, audio_prompt, texts, output_paths=None, verbose=False, max_text_tokens_per_sentence=120,
                   **generation_kwargs):
        self.calls.append(("many", list(texts)))
        if POISON in texts:
            raise ValueError("poisoned cue")
        return [(24000, fake_pcm(t, generation_kwargs)) for t in texts]

    def _synthesize(self, audio_prompt, text, output_path, verbose, max_tokens, gen, fast, bucket_max_size=4):
        self.calls.append(("one", text))
        if text == POISON:
            raise ValueError("poisoned cue")
        return (24000, fake_pcm(text, gen))


class WorkerStub:
    """What a DevicePool worker builds in the CPU tests (``builder="stub_tts:WorkerStub"``)."""

    def __init__(self, cfg_path=None, model_dir=None, is_fp16=True, device="cuda:0"):
        if device == "cuda:7":
            raise RuntimeError("no such device in this test")
        self.device = device

    def infer_many(self, audio_prompt, texts, output_paths=None, verbose=False, max_text_tokens_per_sentence=120,
                   **gen):
        if POISON in texts:
            raise ValueError("poisoned cue")
        if "__die__" in texts:
            import os
            os._exit(3)
        if any("__hang__" in t for t in texts):
            import time
            time.sleep(3600)
        return [(24000, fake_pcm(t, gen)) for t in texts]
