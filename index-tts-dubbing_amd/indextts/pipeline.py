"""Batched IndexTTS hot path: conditioning -> GPT greedy decode -> remove_long_silence -> latent pass
-> BigVGAN2 -> int16 PCM, for many utterances at once on one GPU.

The reference runs this chain one sentence at a time (``IndexTTS.infer``, ``indextts/infer.py:553-631``)
or in buckets of <= 4 (``infer_fast``); here a whole batch (32 by default) shares every launch, and each
utterance's result equals what it produces alone (per-row decode state, per-utterance lengths in the
latent pass and the vocoder).
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .gpt.engine import HipGPT
from .vocoder.bigvgan import HipBigVGAN

HOP = 1024
SR = 24000


def remove_long_silence(codes: np.ndarray, stop: int, silent_token: int = 52, max_consecutive: int = 30):
    """``IndexTTS.remove_long_silence`` (infer.py:132-186) for one row -> kept codes (1-D int64)."""
    hits = np.nonzero(codes == stop)[0]
    n = int(hits[0]) if len(hits) else codes.shape[0]
    if int((codes == silent_token).sum()) > max_consecutive:
        keep, run = [], 0
        for k in range(n):
            if codes[k] != silent_token:
                keep.append(k)
                run = 0
            elif run < 10:
                keep.append(k)
                run += 1
        return codes[keep]
    return codes[:n]


def concat_latents(latent: torch.Tensor, lens: torch.Tensor, spk: torch.Tensor, groups: List[List[int]]):
    """latent [B, T, D] (rows valid up to lens[b]) -> [G, T', D] with group g = time-concatenation of
    its members' valid rows (``torch.cat(items, dim=1)``, infer.py:454)."""
    n = [int(v) for v in lens]
    glen = [sum(n[i] for i in g) for g in groups]
    out = latent.new_zeros(len(groups), max(glen), latent.shape[2])
    for gi, g in enumerate(groups):
        t = 0
        for i in g:
            out[gi, t: t + n[i]] = latent[i, : n[i]]
            t += n[i]
    return out, torch.tensor(glen, dtype=lens.dtype), spk[[g[0] for g in groups]]


class BatchedTTS:
    def __init__(self, gpt_state_dict, bigvgan_state_dict, cfg, device="cuda", dtype: str = "bf16",
                 max_kv: Optional[int] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.gpt = HipGPT(gpt_state_dict, cfg.gpt, device, dtype=dtype, max_kv=max_kv)
        self.vocoder = HipBigVGAN(bigvgan_state_dict, cfg.bigvgan, device)
        self.stop = int(cfg.gpt.stop_mel_token)
        self.stop_text = int(cfg.gpt.stop_text_token)
        self._prompt_cache: Dict[object, tuple] = {}
        self.graph_features = True  # prompt conditioning + ECAPA replayed as a captured graph
        # bf16 product mode: the per-prompt linear layers / 1x1 convs on the bf16 MFMA GEMM (the
        # reference's fp16 mode autocasts them, infer.py:572-586, 613-623); f32 mode stays exact f32
        self.fast_features = dtype == "bf16" and os.environ.get("ITTS_FAST_FEATURES", "1") != "0"
        self._feat_graphs: Dict[tuple, tuple] = {}

    @torch.no_grad()
    def _features(self, m: torch.Tensor):
        """conditioning latents + ECAPA speaker embedding of prompt mels m [n, 100, T]: ~300 small
        PyTorch-ROCm launches, replayed as one captured hipGraph per (n, T) after a warm-up call."""
        fast = self.fast_features
        if not self.graph_features:
            return self.gpt.conditioning(m, fast=fast), self.vocoder.speaker(m.transpose(1, 2), fast=fast)
        key = tuple(m.shape) + (fast,)
        ent = self._feat_graphs.get(key)
        if ent is None:
            static = m.clone()
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):  # warm-up: lets the conv libraries pick their kernels
                self.gpt.conditioning(static, fast=fast), self.vocoder.speaker(static.transpose(1, 2), fast=fast)
            torch.cuda.current_stream(self.device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                c = self.gpt.conditioning(static, fast=fast)
                s = self.vocoder.speaker(static.transpose(1, 2), fast=fast)
            ent = self._feat_graphs[key] = (g, static, c, s)
        g, static, c, s = ent
        static.copy_(m)
        g.replay()
        return c.clone(), s.clone()

    @torch.no_grad()
    def prompt_features(self, mels: Sequence[torch.Tensor], keys: Optional[Sequence[object]] = None):
        """per-prompt conditioning (conds [32, D]) and speaker embedding ([spk_dim]); cached by key."""
        feats: Dict[int, tuple] = {}
        # one evaluation per distinct prompt: a prompt's features must not depend on how many
        # utterances share it in this call (batched-conv rounding differs with the batch size)
        first: Dict[object, int] = {}
        todo = []
        for i in range(len(mels)):
            if keys is None:
                todo.append(i)
            elif keys[i] not in self._prompt_cache and keys[i] not in first:
                first[keys[i]] = i
                todo.append(i)
        by_len: Dict[int, List[int]] = {}  # equal-length prompts share one batched call
        for i in todo:
            by_len.setdefault(int(mels[i].shape[-1]), []).append(i)
        for idx in by_len.values():
            m = torch.cat([mels[i].reshape(1, mels[i].shape[-2], mels[i].shape[-1]) for i in idx], 0).to(self.device)
            c, s = self._features(m)
            for j, i in enumerate(idx):
                feats[i] = (c[j], s[j])
                if keys is not None:
                    self._prompt_cache[keys[i]] = feats[i]
        vals = [feats[i] if i in feats else self._prompt_cache[keys[i]] for i in range(len(mels))]
        return torch.stack([v[0] for v in vals]), torch.stack([v[1] for v in vals])

    @torch.no_grad()
    def synthesize(self, mels: Sequence[torch.Tensor], texts: Sequence[torch.Tensor], max_mel_tokens: int = 600,
                   repetition_penalty: float = 10.0, min_new_tokens: int = 0, keys=None, use_graph: bool = True,
                   timings: Optional[dict] = None, vocoder_groups: Optional[List[List[int]]] = None,
                   pad_to: int = 0, **sampling):
        """mels[b]: prompt log-mel [1, 100, T_b]; texts[b]: token ids [L_b].
        -> (pcm int16 [B, Tmax] on device, sample lengths [B] (cpu), codes list).
        ``timings``: if a dict is given, per-phase wall seconds are accumulated into it (adds syncs).
        ``sampling``: do_sample / temperature / top_k / top_p / seed (HipGPT.generate).
        ``pad_to``: pad the text ids for ``generate`` to at least this length (with the stop id, which
        prepare_gpt_inputs strips -- per-utterance ids unchanged) so that batches of a length bucket share
        one captured decode graph; the latent pass always gets the unpadded ids.
        ``vocoder_groups``: utterance index lists whose latents are concatenated along time before the
        vocoder (``infer_fast`` decodes pairs of sentences as one latent, infer.py:440-458); the pcm /
        lengths then have one row per group (speaker embedding of the group's first member)."""
        import time

        def mark(name, t=[None]):
            if timings is None:
                return
            torch.cuda.synchronize(self.device)
            now = time.perf_counter()
            if t[0] is not None:
                timings[name] = timings.get(name, 0.0) + now - t[0]
            t[0] = now

        mark(None)
        B = len(texts)
        conds, spk = self.prompt_features(mels, keys)
        mark("prompt_features")
        L = max([int(t.numel()) for t in texts] + [int(pad_to)])
        ids = torch.full((B, L), self.stop_text, dtype=torch.long)
        for b, t in enumerate(texts):
            ids[b, : t.numel()] = t.reshape(-1).long()
        codes = self.gpt.generate(conds, ids.to(self.device), max_mel_tokens, repetition_penalty=repetition_penalty,
                                  min_new_tokens=min_new_tokens, use_graph=use_graph, **sampling)
        mark("gpt_generate")
        rows = codes.cpu().numpy()
        self.last_raw_codes = rows  # [B, n] as generated (finished rows padded with the stop token)
        fixed = [torch.from_numpy(remove_long_silence(rows[b], self.stop)) for b in range(B)]
        fixed = [f if f.numel() > 0 else torch.tensor([self.stop]) for f in fixed]  # degenerate: nothing generated
        mark("remove_long_silence")
        latent, lens = self.gpt.latent(conds, [t.reshape(-1) for t in texts], fixed)
        mark("latent_pass")
        if vocoder_groups is not None:
            latent, lens, spk = concat_latents(latent, lens, spk, vocoder_groups)
        _, pcm = self.vocoder.forward(latent, lens, spk)
        mark("vocoder")
        return pcm, (lens.long() * HOP), fixed

    @torch.no_grad()
    def synthesize_many(self, batches: Sequence[tuple], max_mel_tokens: int = 600, repetition_penalty: float = 10.0,
                        min_new_tokens: int = 0, keys=None, front_priority: int = -1, streams=None,
                        overlap: Optional[bool] = None, **sampling):
        """Pipelined ``synthesize`` over several batches [(mels, texts[, {"max_mel_tokens": n,
        "min_new_tokens": m, "pad_to": L}]), ...] (``pad_to`` as in ``synthesize``): the front half (prompt
        features, GPT decode, remove_long_silence) of batch i+1 runs on a high-priority stream while
        the back half (latent pass + vocoder) of batch i runs on a second stream.  The decode step is a
        latency-bound chain of small kernels that leaves most CUs idle; the vocoder's MFMA/HBM-heavy
        launches fill them.  Every batch's results are identical to ``synthesize`` (same kernels,
        same per-row math; only the launch interleaving differs).
        ``overlap`` (default: auto) False runs the batches back to back on one stream: the persistent decode
        layers need every CU, so an overlapped decode runs on the slower launch chain, and when every batch
        would otherwise decode on the persistent layers the serial order is faster (C3, 32 rows: 1455 vs
        1357 audio-s/s); auto overlaps only when some batch decodes on the chain anyway.
        -> list of (pcm int16 [B, Tmax] (device), sample lengths [B] (cpu), codes list); synchronise
        the device (or the current stream) before reading pcm."""
        dev = self.device
        cur = torch.cuda.current_stream(dev)
        if overlap is None:
            beams = int(sampling.get("num_beams", 1) or 1)
            overlap = streams is not None or not all(self.gpt.pl_takes(len(b[1]) * beams, beams > 1) for b in batches)
        if streams is not None:  # caller-made streams (e.g. a CU-masked back stream)
            front, back = streams
        elif not overlap:
            front = back = torch.cuda.Stream(dev)
        else:
            front = torch.cuda.Stream(dev, priority=front_priority)
            back = torch.cuda.Stream(dev)
        front.wait_stream(cur)
        back.wait_stream(cur)
        keep, out = [], []
        for bi, batch in enumerate(batches):
            mels, texts = batch[0], batch[1]
            over = batch[2] if len(batch) > 2 else {}  # per-batch max_mel_tokens / min_new_tokens
            B = len(texts)
            with torch.cuda.stream(front):
                conds, spk = self.prompt_features(mels, None if keys is None else keys[bi])
                L = max([int(t.numel()) for t in texts] + [int(over.get("pad_to", 0))])
                ids = torch.full((B, L), self.stop_text, dtype=torch.long)
                for b, t in enumerate(texts):
                    ids[b, : t.numel()] = t.reshape(-1).long()
                # from the second batch on the back stream may run the previous batch's latent pass and vocoder
                # beside this decode: the persistent decode grid needs every CU at once (gpt_layer.hip), so
                # those decodes run on the launch chain (bit-identical results)
                with self.gpt.launch_chain() if bi > 0 and front is not back else contextlib.nullcontext():
                    codes = self.gpt.generate(conds, ids.to(dev), over.get("max_mel_tokens", max_mel_tokens),
                                              repetition_penalty=repetition_penalty,
                                              min_new_tokens=over.get("min_new_tokens", min_new_tokens), **sampling)
                rows = codes.cpu().numpy()  # syncs the front stream only
            fixed = [torch.from_numpy(remove_long_silence(rows[b], self.stop)) for b in range(B)]
            fixed = [f if f.numel() > 0 else torch.tensor([self.stop]) for f in fixed]
            back.wait_stream(front)
            with torch.cuda.stream(back):
                latent, lens = self.gpt.latent(conds, [t.reshape(-1) for t in texts], fixed)
                _, pcm = self.vocoder.forward(latent, lens, spk)
            keep.append((conds, spk, codes, latent))  # alive until both streams are past them
            out.append((pcm, lens.long() * HOP, fixed))
        cur.wait_stream(back)
        cur.wait_stream(front)
        self._pipeline_keep = keep  # released by the next call (the caller synchronises before reuse)
        return out
