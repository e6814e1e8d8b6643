"""Drop-in ``indextts.infer.IndexTTS`` (reference ``indextts/infer.py:26-660``) on the HIP path.

Same constructor, methods, argument meaning, return values and attributes as the reference, so the
reference's callers (``indextts/cli.py``, ``webui.py``, ``srt_dubbing``'s
``IndexTTSEngine``, which introspects ``inspect.signature(IndexTTS.infer)``, quirk Q9) run unchanged.
What differs is underneath:

* every sentence of one ``infer`` / ``infer_fast`` call is synthesised in ONE batched pass
  (``pipeline.BatchedTTS``: batched GPT prefill + hipGraph decode, batched latent pass, ragged
  batched vocoder) instead of a Python loop over sentences; per-sentence results are unchanged
  because every kernel is row-independent (tests/test_gpu_gpt.py batch-invariance tests);
* ``is_fp16=True`` computes in bf16 (MFMA) with f32 accumulation / residual stream / logits;
  ``is_fp16=False`` runs the exact-f32 verification kernels;
* there is no CPU / MPS path and no silent fallback: without a GPU or without ``libitts_hip.so``
  the constructor raises (the reference fell back to torch, infer.py:97-109);
* decoding: greedy (``do_sample=False, num_beams=1``) reproduces the reference's ids exactly (f32);
  ``do_sample=True`` runs the Temperature/TopK/TopP warpers + multinomial draw on the GPU with a
  device RNG (same distribution, different draws than torch -- statistical parity).  ``num_beams > 1``
  (the reference default: beam sample, 3 beams) runs HF 4.36 beam_search / beam_sample on the GPU
  (gpt_beam.hip; beam search ids bit-exact in f32 mode, beam sample statistical).  An extra ``seed=``
  generation kwarg fixes the device RNG.
"""
from __future__ import annotations

import os
import sys
import time
import warnings
from typing import Dict, List, Optional

import numpy as np
import torch

from .devpool import DevicePool, WorkerError, deal, parse_devices
from .pipeline import HOP, SR, BatchedTTS, remove_long_silence as _rls_row
from .utils.audio import prompt_mel, save_wav_int16
from .utils.config import load_config
from .utils.text import TextNormalizer, TextTokenizer


def _load_state_dict(path: str, key: Optional[str] = None) -> Dict[str, torch.Tensor]:
    """torch.load with ``weights_only=True`` (never unpickles code); unwraps ``{"model": ...}``
    (utils/checkpoint.py:25-27) or the given key (``"generator"`` for BigVGAN, infer.py:112-113)."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if key is not None:
        sd = sd[key]
    elif isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    return sd


def _is_cue(e) -> bool:
    """an object shaped like srt_dubbing's cue (srt_parser.SRTEntry: index, start_time, end_time, text and the
    ``duration`` property the strategies read): a ``str`` text and a numeric duration"""
    return isinstance(getattr(e, "text", None), str) and isinstance(getattr(e, "duration", None), (int, float))


def _is_cue_list(v) -> bool:
    return isinstance(v, (list, tuple)) and len(v) > 1 and all(_is_cue(e) for e in v[:8])


def _caller_cue_texts(text: str, max_depth: int = 8) -> Optional[List[str]]:
    """FALLBACK discovery of the caller's cue list (the explicit hook is ``IndexTTS.prefetch``): the
    texts of the cues from ``text`` on, when ``infer`` runs inside a loop over a list of cue objects.
    srt_dubbing's strategies iterate ``for i, entry in enumerate(entries)`` and call
    ``tts_engine.synthesize(text=entry.text, ...)`` (srt_dubbing/src/strategies/basic_strategy.py:65-74,
    stretch / hq_stretch / adaptive likewise) -> ``IndexTTSEngine.synthesize`` -> ``infer``
    (tts_engines/index_tts_engine.py:45-63).  Kept narrow: in each calling frame
    (innermost first) a local list or tuple of SRT-cue-shaped objects (a ``str`` ``text`` and a numeric
    ``duration``, as ``SRTEntry``) is a candidate (the one named ``entries`` first) only when the same
    frame also holds an ``int`` local that indexes a cue with exactly this text -- the loop counter of
    ``for i, entry in enumerate(entries)``, whatever its name.  None otherwise: then ``infer``
    synthesises this text alone, exactly as the reference does."""
    f = sys._getframe(2)
    try:
        for _ in range(max_depth):
            if f is None:
                return None
            loc = f.f_locals
            cands = sorted(((n != "entries", n) for n, v in loc.items() if _is_cue_list(v)))
            for _, name in cands:
                texts = [e.text for e in loc[name]]
                if text not in texts:
                    continue
                pos = next((v for v in loc.values() if type(v) is int and 0 <= v < len(texts) and texts[v] == text),
                           None)
                if pos is not None:
                    return texts[pos:]
            f = f.f_back
        return None
    finally:
        del f


class IndexTTS:
    MAX_BATCH = 32
    # long-form chunks (infer_many, the cue lookahead): the decode step is latency-bound at 32 rows, so
    # more rows per step raise throughput -- 128 rows decode at 194 ms per 32 rows of 400 codes vs 330
    # for 32 rows alone (profiles/lanes_probe_r02.txt); per-row results do not depend on the chunking
    LONGFORM_BATCH = int(os.environ.get("ITTS_LONGFORM_BATCH", "128"))

    def __init__(self, cfg_path="checkpoints/config.yaml", model_dir="checkpoints", is_fp16=True, device=None,
                 use_cuda_kernel=None):
        if device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("IndexTTS (MI355X build) needs a ROCm GPU; there is no CPU/MPS path")
            device = "cuda:0"
        if not str(device).startswith("cuda"):
            raise RuntimeError(f"device {device!r}: the MI355X build runs on HIP devices ('cuda[:n]') only")
        self.device = str(device)
        self.is_fp16 = bool(is_fp16)
        # more GPUs behind this one object (ITTS_DEVICES="0,1,..." or "all"): worker processes are
        # spawned first so that they load their weights while this process builds its own engine
        self._pool = None
        workers = parse_devices(os.environ.get("ITTS_DEVICES"), torch.cuda.device_count())
        if self.device in workers:
            workers.remove(self.device)  # this process is the listed device's engine
        elif workers and self.device == "cuda" and "cuda:0" in workers:
            workers.remove("cuda:0")
        # the persistent decode layer needs every one of its workgroups resident at once: on a GPU that
        # several engines share (ITTS_DEVICES listing one device twice -- the tests' stand-in for two
        # GPUs) their grids could each hold part of the CUs, so those engines use the launch chain
        # (bit-identical results)
        every = [self.device] + workers
        shared = {d for d in every if every.count(d) > 1}
        if workers:
            self._pool = DevicePool(cfg_path, model_dir, self.is_fp16, workers, no_pl=shared)
        # the fused anti-alias activation is always the HIP kernel here; kept for API compatibility
        self.use_cuda_kernel = use_cuda_kernel is None or bool(use_cuda_kernel)
        self.cfg = load_config(cfg_path)
        self.model_dir = model_dir
        self.dtype = torch.bfloat16 if self.is_fp16 else None
        self.stop_mel_token = self.cfg.gpt.stop_mel_token

        self.gpt_path = os.path.join(model_dir, self.cfg.gpt_checkpoint)
        self.bigvgan_path = os.path.join(model_dir, self.cfg.bigvgan_checkpoint)
        gpt_sd = _load_state_dict(self.gpt_path)
        print(">> GPT weights restored from:", self.gpt_path)
        bv_sd = _load_state_dict(self.bigvgan_path, "generator")
        print(">> bigvgan weights restored from:", self.bigvgan_path)
        self.engine = BatchedTTS(gpt_sd, bv_sd, self.cfg, self.device, dtype="bf16" if self.is_fp16 else "f32")
        self.gpt, self.bigvgan = self.engine.gpt, self.engine.vocoder
        if self.device in shared:
            self.gpt.pl = False
        del gpt_sd, bv_sd

        self.bpe_path = os.path.join(model_dir, self.cfg.dataset["bpe_model"])
        self.normalizer = TextNormalizer()
        self.normalizer.load()
        print(">> TextNormalizer loaded")
        self.tokenizer = TextTokenizer(self.bpe_path, self.normalizer)
        print(">> bpe model loaded from:", self.bpe_path)
        self.cache_audio_prompt = None
        self.cache_cond_mel = None
        self.gr_progress = None
        self.model_version = self.cfg.version if "version" in self.cfg else None

    # ------------------------------------------------------------------ host helpers (reference API)
    def remove_long_silence(self, codes: torch.Tensor, silent_token=52, max_consecutive=30):
        """infer.py:132-186: cut each row at its first stop token; rows with > max_consecutive silent
        tokens keep at most 10 consecutive ones.  -> (codes [B, n], code_lens [B])"""
        rows, lens, fixed = [], [], False
        arr = codes.detach().cpu().numpy()
        for r in arr:
            kept = _rls_row(r, int(self.stop_mel_token), silent_token, max_consecutive)
            hit = np.nonzero(r == self.stop_mel_token)[0]
            n_cut = int(hit[0]) if len(hit) else r.shape[0]
            if int((r == silent_token).sum()) > max_consecutive:
                fixed = True
            rows.append(kept)
            lens.append(kept.shape[0] if int((r == silent_token).sum()) > max_consecutive else n_cut)
        if fixed:
            width = max(x.shape[0] for x in rows)
            out = np.full((len(rows), width), self.stop_mel_token, dtype=arr.dtype)
            for i, x in enumerate(rows):
                out[i, : x.shape[0]] = x
            codes = torch.from_numpy(out).to(codes.device)
        mx = max(lens)
        if mx < codes.shape[1]:
            codes = codes[:, :mx]
        return codes, torch.tensor(lens, dtype=torch.long, device=codes.device)

    def bucket_sentences(self, sentences, bucket_max_size=4) -> List[List[Dict]]:
        """infer.py:188-243: sort by length, open a new bucket when a sentence reaches 1.5x the running
        bucket median or the bucket is full, then fold singleton buckets into open buckets."""
        items = [{"idx": i, "sent": s, "len": len(s)} for i, s in enumerate(sentences)]
        if len(items) <= bucket_max_size:
            return [items]
        buckets: List[List[Dict]] = []
        median = 0
        for it in sorted(items, key=lambda d: d["len"]):
            if it["len"] == 0:
                print(">> skip empty sentence")
                continue
            if not buckets or it["len"] >= int(median * 1.5) or len(buckets[-1]) >= bucket_max_size:
                buckets.append([it])
                median = it["len"]
            else:
                buckets[-1].append(it)
                median = buckets[-1][len(buckets[-1]) // 2]["len"]
        multi = [b for b in buckets if len(b) > 1]
        singles = [b[0] for b in buckets if len(b) == 1]
        for b in multi:
            if not singles:
                break
            if len(b) < bucket_max_size:
                b.append(singles.pop(0))
        multi.extend(singles[i: i + bucket_max_size] for i in range(0, len(singles), bucket_max_size))
        return multi

    def pad_tokens_cat(self, tokens: List[torch.Tensor]) -> torch.Tensor:
        """infer.py:245-262: v1.5+ right-pads [1, n] rows with stop_text; older versions pad up to 8
        stop_text then start_text."""
        width = max(t.shape[-1] for t in tokens)
        stop, start = self.cfg.gpt.stop_text_token, self.cfg.gpt.start_text_token
        out = torch.empty(len(tokens), width, dtype=tokens[0].dtype, device=tokens[0].device)
        for i, t in enumerate(tokens):
            row = t.reshape(-1)
            n = row.numel()
            out[i, :n] = row
            if self.model_version and self.model_version >= 1.5:
                out[i, n:] = stop
            else:
                k = min(8, width - n)
                out[i, n: n + k] = stop
                out[i, n + k:] = start
        return out

    def torch_empty_cache(self):
        try:
            torch.cuda.empty_cache()
        except Exception:
            pass

    def _set_gr_progress(self, value, desc):
        if self.gr_progress is not None:
            self.gr_progress(value, desc=desc)

    # ------------------------------------------------------------------ shared driver
    def _prompt(self, audio_prompt):
        if self.cache_cond_mel is None or self.cache_audio_prompt != audio_prompt:
            cond_mel = prompt_mel(audio_prompt, self.device)  # resample + log-mel on the GPU
            self.cache_audio_prompt = audio_prompt
            self.cache_cond_mel = cond_mel
            self.engine._prompt_cache.clear()  # conditioning / speaker embedding follow the mel cache
        return self.cache_cond_mel

    @staticmethod
    def _decoding(kw: dict, max_tok_default=600):
        do_sample = kw.pop("do_sample", True)
        top_p = kw.pop("top_p", 0.8)
        top_k = kw.pop("top_k", 30)
        temperature = kw.pop("temperature", 1.0)
        length_penalty = kw.pop("length_penalty", 0.0)
        num_beams = kw.pop("num_beams", 3)
        repetition_penalty = kw.pop("repetition_penalty", 10.0)
        max_mel_tokens = kw.pop("max_mel_tokens", max_tok_default)
        min_new_tokens = kw.pop("min_new_tokens", 0)
        seed = kw.pop("seed", None)
        kw.pop("num_return_sequences", None)
        # inference_speech's own defaults (gpt/model.py:655-656): typical sampling off (typical_mass then unused) and
        # HF generate's use_cache=True are what the HIP decode does anyway; only the settings it cannot honour warn
        if not kw.get("typical_sampling", False):
            kw.pop("typical_sampling", None)
            kw.pop("typical_mass", None)
        if kw.get("use_cache", True):
            kw.pop("use_cache", None)
        if kw:  # e.g. typical_sampling=True, no_repeat_ngram_size (gpt/model.py:655-708 -> HF generate)
            warnings.warn(f"ignored generation kwargs: {sorted(kw)} -- the HIP decode honours do_sample, top_p, "
                          "top_k, temperature, length_penalty, num_beams, repetition_penalty, max_mel_tokens, "
                          "min_new_tokens, seed (INTEGRATION.md §2); the reference would pass the rest to "
                          "inference_speech / HF generate", RuntimeWarning)
        num_beams = int(num_beams or 1)
        if num_beams > 16:
            raise ValueError("HIP beam search supports num_beams <= 16")
        smp = {}
        if num_beams > 1:
            smp = dict(num_beams=num_beams, length_penalty=float(length_penalty or 0.0))
        if do_sample:
            top_k = int(top_k or 0)
            smp.update(do_sample=True, temperature=float(temperature), top_k=top_k,
                       top_p=1.0 if top_p is None else float(top_p), seed=seed)
        return dict(max_mel_tokens=int(max_mel_tokens), repetition_penalty=float(repetition_penalty),
                    min_new_tokens=int(min_new_tokens), **smp)

    def _run(self, cond_mel, sent_ids: List[torch.Tensor], dec: dict, groups=None):
        """all sentences (chunks of MAX_BATCH) through the batched HIP pipeline -> (pcm rows, codes)."""
        pcm_rows, codes_all = [], []
        keys = [("prompt", self.cache_audio_prompt)]
        B = self.MAX_BATCH
        for c0 in range(0, len(sent_ids), B):
            chunk = sent_ids[c0: c0 + B]
            g = None
            if groups is not None:  # groups never straddle a chunk boundary (pairs, B even)
                g = [[i - c0 for i in grp] for grp in groups if c0 <= grp[0] < c0 + B]
            pcm, n, fixed = self.engine.synthesize([cond_mel] * len(chunk), chunk, keys=keys * len(chunk),
                                                   vocoder_groups=g, **dec)
            pcm = pcm.cpu()
            pcm_rows += [pcm[i, : int(n[i])] for i in range(pcm.shape[0])]
            codes_all += fixed
            raw = self.engine.last_raw_codes
            self._hit_limit = self._hit_limit or bool((raw != self.stop_mel_token).all(axis=1).any())
        return pcm_rows, codes_all

    def _finish(self, pcm_rows, output_path, t0, cond_frames, label=""):
        wav = torch.cat(pcm_rows) if pcm_rows else torch.zeros(0, dtype=torch.int16)
        end = time.perf_counter()
        wav_len = wav.shape[0] / SR
        print(f">> Reference audio length: {cond_frames * 256 / SR:.2f} seconds")
        print(f">> Total {label}inference time: {end - t0:.2f} seconds")
        print(f">> Generated audio length: {wav_len:.2f} seconds")
        if wav_len > 0:
            print(f">> {'[fast] ' if label else ''}RTF: {(end - t0) / wav_len:.4f}")
        data = wav.numpy().astype(np.int16).reshape(-1, 1)
        if output_path:
            if os.path.isfile(output_path):
                os.remove(output_path)
                print(">> remove old wav file:", output_path)
            if os.path.dirname(output_path) != "":
                os.makedirs(os.path.dirname(output_path), exist_ok=True)
            save_wav_int16(output_path, data, SR)
            print(">> wav file saved to:", output_path)
            return output_path
        return (SR, data)

    def _warn_truncated(self, codes_raw_hit_limit, max_mel_tokens, max_text_tokens_per_sentence):
        if codes_raw_hit_limit:
            warnings.warn(f"WARN: generation stopped due to exceeding `max_mel_tokens` ({max_mel_tokens}). "
                          f"Consider reducing `max_text_tokens_per_sentence`({max_text_tokens_per_sentence}) "
                          "or increasing `max_mel_tokens`.", category=RuntimeWarning)

    def _synthesize(self, audio_prompt, text, output_path, verbose, max_tokens, gen, fast, bucket_max_size=4):
        print(">> start fast inference..." if fast else ">> start inference...")
        self._set_gr_progress(0, "start fast inference..." if fast else "start inference...")
        if verbose:
            print(f"origin text:{text}")
        t0 = time.perf_counter()
        cond_mel = self._prompt(audio_prompt)
        self._set_gr_progress(0.1, "text processing...")
        tokens = self.tokenizer.tokenize(text)
        sentences = self.tokenizer.split_sentences(tokens, max_tokens)
        if verbose:
            print("text token count:", len(tokens))
            print("sentences count:", len(sentences))
            print("max_text_tokens_per_sentence:", max_tokens)
            print(*sentences, sep="\n")
        dec = self._decoding(dict(gen))
        order = list(range(len(sentences)))
        if fast:  # bucketing only decides which sentences share a GPT batch in the reference; every
            # sentence is batched here, so it only drops empty sentences (as the reference does)
            order = [d["idx"] for b in self.bucket_sentences(sentences, bucket_max_size) for d in b]
            order.sort()
        ids = [torch.tensor(self.tokenizer.convert_tokens_to_ids(sentences[i]), dtype=torch.int32) for i in order]
        if not ids:
            return self._finish([], output_path, t0, cond_mel.shape[-1], "fast " if fast else "")
        groups = None
        if fast:  # BigVGAN decodes the latents of consecutive sentence pairs as one sequence
            groups = [list(range(i, min(i + 2, len(ids)))) for i in range(0, len(ids), 2)]
        self._set_gr_progress(0.2, "gpt inference speech...")
        self._hit_limit = False
        pcm_rows, codes = self._run(cond_mel, ids, dec, groups)
        self._warn_truncated(self._hit_limit, dec["max_mel_tokens"], max_tokens)
        self._set_gr_progress(0.9, "save audio...")
        return self._finish(pcm_rows, output_path, t0, cond_mel.shape[-1], "fast " if fast else "")

    # ------------------------------------------------------------------ public API
    def infer_fast(self, audio_prompt, text, output_path, verbose=False, max_text_tokens_per_sentence=100,
                   sentences_bucket_max_size=4, **generation_kwargs):
        """infer.py:278-497 (sentence pairs vocoded together; one batched GPT pass for all sentences)."""
        return self._synthesize(audio_prompt, text, output_path, verbose, max_text_tokens_per_sentence,
                                generation_kwargs, fast=True, bucket_max_size=sentences_bucket_max_size)

    def infer(self, audio_prompt, text, output_path, verbose=False, max_text_tokens_per_sentence=120,
              **generation_kwargs):
        """infer.py:500-660 -> output_path (16-bit PCM 24 kHz wav written) or (24000, int16 [T, 1]).

        Cross-call batching for callers that loop over cues one ``infer`` at a time (srt_dubbing's
        strategies -> ``IndexTTSEngine.synthesize``, unchanged): a result prefetched by ``prefetch``
        (or by the lookahead below) for the same prompt, text and arguments is returned instead of a
        new synthesis."""
        key = self._ahead_key(audio_prompt, max_text_tokens_per_sentence, generation_kwargs)
        hit = self._take_ahead(key, text)
        if hit is None and self._lookahead_ok(key, text):
            upcoming = _caller_cue_texts(text)
            if upcoming and len(upcoming) > 1:
                window = upcoming[: self.LOOKAHEAD * self.n_devices]
                try:
                    self.prefetch(audio_prompt, window, max_text_tokens_per_sentence, **generation_kwargs)
                except Exception as e:  # noqa: BLE001 -- e.g. one bad cue: never fail the whole window
                    # its cues are synthesised one call at a time from now on, so an error hits only the
                    # cue that causes it (the reference's behaviour: basic_strategy.py:86-97 writes silence)
                    warnings.warn(f"lookahead batch of {len(window)} cues failed ({e!r}); those cues are "
                                  "synthesised one call at a time", RuntimeWarning)
                    self._ahead_state()["bad"].update(window)
                hit = self._take_ahead(key, text)
        self._ahead_state()["last"] = (text, key)
        if hit is not None:
            return self._deliver(hit, output_path)
        return self._synthesize(audio_prompt, text, output_path, verbose, max_text_tokens_per_sentence,
                                generation_kwargs, fast=False)

    # ------------------------------------------------------------------ cross-call batching
    # Cues synthesised ahead per device when ``infer`` is called from inside a loop over a cue list
    # (0: off).  The explicit hook is ``prefetch``; the frame walk (_caller_cue_texts) is the fallback
    # that batches the unchanged srt_dubbing caller.
    LOOKAHEAD = int(os.environ.get("ITTS_LOOKAHEAD", "128"))
    AHEAD_CAP_WINDOWS = 4  # prefetched results kept: at most this many windows (oldest dropped)

    @property
    def n_devices(self) -> int:
        return 1 + (len(self._pool.alive()) if self.__dict__.get("_pool") is not None else 0)

    def _ahead_state(self):
        st = self.__dict__.get("_ahead_st")
        if st is None:
            # ahead: (key, text) -> FIFO of results; win: key -> [issued, consumed] of its last window;
            # recent: keys of the last windows, oldest first; bad: texts of windows that failed;
            # last: (text, key) of the previous call
            st = self.__dict__["_ahead_st"] = {"ahead": {}, "win": {}, "recent": [], "bad": set(), "last": None}
        return st

    @property
    def _ahead(self):
        return self._ahead_state()["ahead"]

    def _ahead_key(self, audio_prompt, max_tokens, gen):
        """None for a prompt that is not a path (no cross-call reuse: an object's id can be recycled)."""
        if not isinstance(audio_prompt, str):
            return None
        try:
            mtime = os.path.getmtime(audio_prompt)
        except OSError:
            mtime = None
        return (audio_prompt, mtime, int(max_tokens), tuple(sorted((k, repr(v)) for k, v in gen.items())))

    def _lookahead_ok(self, key, text) -> bool:
        """Batch ahead only for a stable argument set: not for a path-less prompt, not for a text whose
        window failed, not when the same text was just requested with other arguments (a duration
        search varying length_penalty per attempt: each attempt is one call, as in the reference), and
        not once the last three windows went mostly unused (< 1/4 of their results taken)."""
        st = self._ahead_state()
        if key is None or self.LOOKAHEAD <= 0 or text in st["bad"] or st.get("off_all"):
            return False
        last = st["last"]
        if last is not None and last[0] == text and last[1] != key:
            return False
        recent = [st["win"][k] for k in st["recent"][-3:] if k in st["win"]]
        if len(recent) == 3 and all(w[0] >= 4 and 4 * w[1] < w[0] for w in recent):
            # the last three windows went mostly unused (a caller that changes its arguments per cue):
            # batching ahead only multiplies the work -- off for this object from now on
            warnings.warn("cue lookahead switched off: prefetched results went unused", RuntimeWarning)
            st["off_all"] = True
            return False
        return True

    def _take_ahead(self, key, text):
        if key is None:
            return None
        st = self._ahead_state()
        q = st["ahead"].get((key, text))
        if not q:
            return None
        res = q.pop(0)  # one result per call: a repeated call synthesises anew (new draws when sampling)
        if not q:
            del st["ahead"][(key, text)]
        w = st["win"].get(key)
        if w is not None:
            w[1] += 1
        return res

    def prefetch(self, audio_prompt, texts, max_text_tokens_per_sentence=120, **generation_kwargs):
        """Synthesise ``texts`` now, all sentences of all texts batched (``infer_many``; with
        ITTS_DEVICES, dealt over this process's GPU and the worker GPUs), and keep one result per
        occurrence for the ``infer`` calls that follow with the same prompt (a path), text and
        arguments.  Deterministic decoding (``do_sample=False``): each result equals what that
        ``infer`` call would have computed (rows never interact; tests/test_gpu_lookahead.py, and
        tests/test_gpu_longform.py::test_two_engines_one_gpu_equal_per_call: two processes on one GPU,
        short rows); with sampling it is an independent draw from the same distribution, as a fresh call would be.  Results of an earlier window for the same arguments
        that the caller has moved past are dropped."""
        key = self._ahead_key(audio_prompt, max_text_tokens_per_sentence, generation_kwargs)
        if key is None:
            return
        st = self._ahead_state()
        ahead = st["ahead"]
        window = set(texts)
        for k in [k for k in ahead if k[0] == key and k[1] not in window]:
            del ahead[k]  # behind the caller
        need, have = [], {}
        for t in texts:
            if t in st["bad"]:
                continue
            have[t] = have.get(t, len(ahead.get((key, t), [])))
            if have[t] > 0:
                have[t] -= 1
            else:
                need.append(t)
        if not need:
            return
        res = self._infer_many_devices(audio_prompt, need, max_text_tokens_per_sentence, generation_kwargs)
        for t, r in zip(need, res):
            ahead.setdefault((key, t), []).append(r)
        st["win"][key] = [len(need), 0]
        st["recent"] = [k for k in st["recent"] if k != key][-7:] + [key]
        for k in [k for k in st["win"] if k not in st["recent"]]:
            del st["win"][k]
        cap = self.AHEAD_CAP_WINDOWS * max(self.LOOKAHEAD, 1) * self.n_devices
        while sum(len(q) for q in ahead.values()) > cap:
            del ahead[next(iter(ahead))]  # oldest first

    def _infer_many_devices(self, audio_prompt, texts, max_tokens, gen):
        """``infer_many`` over this process's engine and the live workers (longest texts first onto the
        least-loaded device); a failed worker's share is synthesised here."""
        pool = self.__dict__.get("_pool")
        alive = pool.alive() if pool is not None else []
        if not alive:
            return self.infer_many(audio_prompt, texts, None, False, max_tokens, **gen)
        costs = [max(1, len(self.tokenizer.tokenize(t))) for t in texts]
        bins = deal(costs, 1 + len(alive))
        tickets = []
        for wi, share in zip(alive, bins[1:]):
            if share:
                try:
                    tickets.append((share, pool.submit(wi, audio_prompt, [texts[i] for i in share], max_tokens, gen)))
                except WorkerError:
                    bins[0] = sorted(bins[0] + share)
        out = [None] * len(texts)
        err = None
        try:
            if bins[0]:
                for i, r in zip(bins[0], self.infer_many(audio_prompt, [texts[i] for i in bins[0]], None, False,
                                                         max_tokens, **gen)):
                    out[i] = r
        except Exception as e:  # noqa: BLE001 -- collect the workers' replies first (keeps the pipes in step)
            err = e
        redo = []
        for share, ticket in tickets:
            try:
                for i, r in zip(share, pool.result(ticket)):
                    out[i] = r
            except WorkerError as e:
                warnings.warn(f"{e}; its {len(share)} cue(s) are synthesised on {self.device}", RuntimeWarning)
                redo += share
        if err is not None:
            raise err
        if redo:
            for i, r in zip(redo, self.infer_many(audio_prompt, [texts[i] for i in redo], None, False, max_tokens,
                                                  **gen)):
                out[i] = r
        return out

    def close(self):
        """Stop the worker processes (ITTS_DEVICES); also run at interpreter exit."""
        pool = self.__dict__.get("_pool")
        if pool is not None:
            self._pool = None
            pool.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    @staticmethod
    def _deliver(res, output_path):
        sr, data = res
        if not output_path:
            return (sr, data)
        if os.path.isfile(output_path):
            os.remove(output_path)
        if os.path.dirname(output_path) != "":
            os.makedirs(os.path.dirname(output_path), exist_ok=True)
        save_wav_int16(output_path, data, sr)
        print(">> wav file saved to:", output_path)
        return output_path


    def infer_many(self, audio_prompt, texts, output_paths=None, verbose=False, max_text_tokens_per_sentence=120,
                   **generation_kwargs):
        """Long-form / many-cue entry point (not in the reference): ``infer`` for every
        text in ``texts`` with one shared prompt, all sentences of all texts batched together
        (length-sorted chunks of LONGFORM_BATCH) and streamed through the pipelined driver
        (``BatchedTTS.synthesize_many``: GPT decode of chunk i+1 overlapped with the latent pass +
        vocoder of chunk i).  Per text the result equals ``infer(audio_prompt, text, output_path,
        ...)`` -- a path (wav written) or ``(24000, int16 [T, 1])``; returns the list in order."""
        paths = list(output_paths) if output_paths is not None else [None] * len(texts)
        assert len(paths) == len(texts), "one output path (or None) per text"
        t0 = time.perf_counter()
        cond_mel = self._prompt(audio_prompt)
        dec = self._decoding(dict(generation_kwargs))
        sent_ids, owner = [], []
        for ti, text in enumerate(texts):
            sentences = self.tokenizer.split_sentences(self.tokenizer.tokenize(text), max_text_tokens_per_sentence)
            for sent in sentences:
                sent_ids.append(torch.tensor(self.tokenizer.convert_tokens_to_ids(sent), dtype=torch.int32))
                owner.append(ti)
        order = sorted(range(len(sent_ids)), key=lambda i: -len(sent_ids[i]))
        batches, chunks = [], []
        keys = []
        for c0 in range(0, len(order), self.LONGFORM_BATCH):
            idx = order[c0: c0 + self.LONGFORM_BATCH]
            chunks.append(idx)
            batches.append(([cond_mel] * len(idx), [sent_ids[i].to(self.device) for i in idx]))
            keys.append([("prompt", self.cache_audio_prompt)] * len(idx))
        rows = [None] * len(sent_ids)
        self._hit_limit = False
        if batches:
            res = self.engine.synthesize_many(batches, keys=keys, **dec)
            torch.cuda.synchronize(self.device)
            for idx, (pcm, n, _) in zip(chunks, res):
                pcm = pcm.cpu()
                for j, i in enumerate(idx):
                    rows[i] = pcm[j, : int(n[j])]
        if verbose:
            print(f">> infer_many: {len(texts)} texts, {len(sent_ids)} sentences, {len(batches)} chunks")
        out = []
        for ti in range(len(texts)):
            mine = [rows[i] for i in range(len(sent_ids)) if owner[i] == ti]
            out.append(self._finish(mine, paths[ti], t0, cond_mel.shape[-1]))
        return out


if __name__ == "__main__":  # pragma: no cover
    from .cli import main
    sys.exit(main())
