"""ORACLE (test infrastructure only -- never imported by the product path).

CPU fp32 restatement of the IndexTTS GPT speech-token path, written from the reference's math:
prefill / KV-cached decode of the GPT-2 core, repetition-penalised greedy token selection,
``remove_long_silence`` and the teacher-forced latent pass.  Used by ``tests/`` as the checker
for the HIP path, by ``__graft_entry__.smoke()`` and by ``bench.py``'s ``cpu_baseline`` leg.

Reference anchors (paths relative to the reference tree; ``HF:`` = transformers GPT-2, the
third-party dependency the reference pins at 4.36.2, ``setup.py:50``):
  * prepare_gpt_inputs (strip ids 0/1, [0]+ids+[1], left zero-pad, mask)  gpt/model.py:591-654
  * prefill embedding = [cond;text] ++ mel_emb(8192)+mel_pos[0]         gpt/model.py:139-150
  * decode embedding mel_emb(tok) + mel_pos[mask_len - s]  (quirk Q1)   gpt/model.py:151-155
  * GPT-2 block: LN -> c_attn -> causal/padded SDPA (scale 1/8) -> c_proj -> +res -> LN -> c_fc ->
    gelu_tanh -> c_proj -> +res    HF:modeling_gpt2.py:54-72,185-306 ; wpe == 0 (gpt/model.py:17-18)
  * ln_f then final_norm then mel_head (quirk Q5)                       HF:modeling_gpt2.py:620; gpt/model.py:48,180
  * repetition penalty over all ids incl. fake prefix (Q4); fp32 logits; first-index argmax;
    finished rows padded with 8193                                      HF:generation/logits_process.py:409-412, utils.py:2894-2925
  * remove_long_silence                                                  infer.py:132-186
  * latent pass (teacher forced, positions 0..n+1, drop last 2)         gpt/model.py:521-578, 462-477
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

NEG = torch.finfo(torch.float32).min


def _f32(sd: Dict[str, object]) -> Dict[str, torch.Tensor]:
    return {k: torch.as_tensor(v).float() if torch.as_tensor(v).is_floating_point() else torch.as_tensor(v)
            for k, v in sd.items()}


class GPTOracle:
    def __init__(self, sd, cfg_gpt, sd_decode=None):
        """``sd``: the weights every pass uses; ``sd_decode`` (optional): other weights for the KV-cached
        decode steps only (tests: the bf16 product path stores its prefill and decode GEMM weights
        differently -- rounded W vs rounded diag(ln.g) W, tests/parity_util.py ``bf16_effective_gpt_sds``)."""
        self.sd = _f32(sd)
        self.sd_dec = self.sd if sd_decode is None else _f32(sd_decode)
        g = cfg_gpt
        self.D, self.L, self.H = int(g.model_dim), int(g.layers), int(g.heads)
        self.hd = self.D // self.H
        self.start_text, self.stop_text = int(g.start_text_token), int(g.stop_text_token)
        self.start_mel, self.stop_mel = int(g.start_mel_token), int(g.stop_mel_token)

    # ---------------- inputs ----------------
    def prepare_inputs(self, conds: torch.Tensor, text_ids: torch.Tensor):
        """conds [1|B, 32, D], text_ids [B, L] -> emb [B, s, D], mask [B, s+1] (1 = attend)."""
        sd = self.sd
        B, L = text_ids.shape
        ncond = conds.shape[1]
        s = ncond + L + 2
        emb = torch.zeros(B, s, self.D)
        mask = torch.ones(B, s + 1, dtype=torch.long)
        for i in range(B):
            row = text_ids[i].long()
            row = row[(row != self.stop_text) & (row != self.start_text)]
            row = torch.cat([torch.tensor([self.start_text]), row, torch.tensor([self.stop_text])])
            te = sd["text_embedding.weight"][row] + sd["text_pos_embedding.emb.weight"][: row.numel()]
            c = conds[0] if conds.shape[0] == 1 else conds[i]
            pad = L + 2 - row.numel()
            emb[i, pad:] = torch.cat([c.float(), te], 0)
            mask[i, :pad] = 0
        return emb, mask

    # ---------------- GPT-2 core ----------------
    def _block(self, i, x, kv, attn_bias, sd=None):
        sd, H, hd = sd if sd is not None else self.sd, self.H, self.hd
        p = f"gpt.h.{i}"
        B, T, D = x.shape
        h = F.layer_norm(x, (D,), sd[p + ".ln_1.weight"], sd[p + ".ln_1.bias"], 1e-5)
        qkv = torch.addmm(sd[p + ".attn.c_attn.bias"], h.reshape(-1, D), sd[p + ".attn.c_attn.weight"]).view(B, T, 3, H, hd)
        q, k, v = (qkv[:, :, j].transpose(1, 2) for j in range(3))
        if kv is not None:
            if kv[i] is not None:
                k = torch.cat([kv[i][0], k], 2)
                v = torch.cat([kv[i][1], v], 2)
            kv[i] = (k, v)
        att = (q @ k.transpose(-1, -2)) * (1.0 / math.sqrt(hd)) + attn_bias
        o = (torch.softmax(att, -1) @ v).transpose(1, 2).reshape(B * T, D)
        x = x + torch.addmm(sd[p + ".attn.c_proj.bias"], o, sd[p + ".attn.c_proj.weight"]).view(B, T, D)
        h = F.layer_norm(x, (D,), sd[p + ".ln_2.weight"], sd[p + ".ln_2.bias"], 1e-5)
        f = F.gelu(torch.addmm(sd[p + ".mlp.c_fc.bias"], h.reshape(-1, D), sd[p + ".mlp.c_fc.weight"]), approximate="tanh")
        return x + torch.addmm(sd[p + ".mlp.c_proj.bias"], f, sd[p + ".mlp.c_proj.weight"]).view(B, T, D)

    def core(self, x, attn_bias, kv=None, sd=None):
        sd = self.sd if sd is None else sd
        for i in range(self.L):
            x = self._block(i, x, kv, attn_bias, sd)
        return F.layer_norm(x, (self.D,), sd["gpt.ln_f.weight"], sd["gpt.ln_f.bias"], 1e-5)

    def head(self, h, sd=None):
        sd = self.sd if sd is None else sd
        h = F.layer_norm(h, (self.D,), sd["final_norm.weight"], sd["final_norm.bias"], 1e-5)
        return F.linear(h, sd["mel_head.weight"], sd["mel_head.bias"])

    @staticmethod
    def _bias(mask_keys: torch.Tensor, q_len: int):
        """additive [B, 1, q_len, K] bias: causal over the last q_len keys + key padding."""
        B, K = mask_keys.shape
        qpos = torch.arange(K - q_len, K)[:, None]
        causal = torch.arange(K)[None, :] <= qpos
        ok = causal[None] & mask_keys.bool()[:, None, :]
        return torch.where(ok, 0.0, NEG)[:, None]

    # ---------------- token selection ----------------
    @staticmethod
    def penalize(logits: torch.Tensor, seen: torch.Tensor, penalty: float):
        """``RepetitionPenaltyLogitsProcessor``: x<0 ? x*p : x/p at every id already in the sequence."""
        pen = torch.where(logits < 0, logits * penalty, logits / penalty)
        return torch.where(seen, pen, logits)

    def generate(self, conds, text_ids, max_new_tokens: int, repetition_penalty: float = 10.0,
                 min_new_tokens: int = 0, return_trace: bool = False):
        """Greedy decode (do_sample=False, num_beams=1).  -> codes [B, n] (finished rows padded 8193)."""
        emb, mask = self.prepare_inputs(conds, text_ids)
        B, s, D = emb.shape
        sd = self.sd
        V = sd["mel_head.weight"].shape[0]
        start = sd["mel_embedding.weight"][self.start_mel] + sd["mel_pos_embedding.emb.weight"][0]
        x = torch.cat([emb, start.expand(B, 1, D)], 1)
        kv: List[Optional[tuple]] = [None] * self.L
        h = self.core(x, self._bias(mask, s + 1), kv)
        logits = self.head(h[:, -1])
        seen = torch.zeros(B, V, dtype=torch.bool)
        seen[:, 1] = True  # the fake prefix ids (gpt/model.py:645-653)
        seen[:, self.start_mel] = True
        done = torch.zeros(B, dtype=torch.bool)
        out, trace = [], []
        for step in range(max_new_tokens):
            sc = self.penalize(logits, seen, repetition_penalty)
            if step < min_new_tokens:
                sc[:, self.stop_mel] = float("-inf")
            if return_trace:
                top2 = torch.topk(sc, 2, dim=-1)
                trace.append((sc.clone(), top2.values[:, 0] - top2.values[:, 1]))
            nxt = torch.argmax(sc, dim=-1)
            nxt = torch.where(done, torch.full_like(nxt, self.stop_mel), nxt)
            out.append(nxt)
            seen[torch.arange(B), nxt] = True
            done |= nxt == self.stop_mel
            if bool(done.all()):
                break
            mask = torch.cat([mask, torch.ones(B, 1, dtype=mask.dtype)], 1)
            pos = mask.shape[1] - s  # quirk Q1: position j+1 for the j-th fed-back token (j >= 1)
            e = sd["mel_embedding.weight"][nxt] + sd["mel_pos_embedding.emb.weight"][pos]
            h = self.core(e[:, None], self._bias(mask, 1), kv, self.sd_dec)
            logits = self.head(h[:, -1], self.sd_dec)
        codes = torch.stack(out, 1)
        return (codes, trace) if return_trace else codes

    # ---------------- beam search / beam sample (HF 4.36 semantics) ----------------
    @staticmethod
    def warp(sc: torch.Tensor, temperature: float, top_k: int, top_p: float, min_keep: int):
        """Temperature -> TopK -> TopP warpers (HF:generation/logits_process.py TemperatureLogitsWarper,
        TopKLogitsWarper, TopPLogitsWarper), row-wise; min_keep = 2 under beams (HF 4.36
        ``_get_logits_warper``: eos is a single id)."""
        if temperature != 1.0:
            sc = sc / temperature
        if top_k:
            k = min(max(top_k, min_keep), sc.shape[-1])
            kth = torch.topk(sc, k, dim=-1).values[..., -1:]
            sc = sc.masked_fill(sc < kth, float("-inf"))
        if top_p < 1.0:
            srt, idx = torch.sort(sc, descending=False, dim=-1)
            cum = srt.softmax(-1).cumsum(-1)
            rem = cum <= (1 - top_p)
            rem[..., -min_keep:] = False
            sc = sc.masked_fill(rem.scatter(-1, idx, rem), float("-inf"))
        return sc

    def generate_beam(self, conds, text_ids, max_new_tokens: int, num_beams: int = 3,
                      repetition_penalty: float = 10.0, length_penalty: float = 0.0, min_new_tokens: int = 0,
                      do_sample: bool = False, temperature: float = 1.0, top_k: int = 0, top_p: float = 1.0,
                      generator: Optional[torch.Generator] = None, copies: int = 1, trace: Optional[list] = None):
        """``generate(num_beams=K)`` as transformers 4.36 runs it for ``inference_speech``
        (gpt/model.py:698-703): ``beam_search`` (do_sample=False) or ``beam_sample`` (do_sample=True)
        with ``BeamSearchScorer`` (HF:generation/beam_search.py process / finalize, BeamHypotheses
        add / is_done; early_stopping=False, one returned sequence per input).

        * step scores = log_softmax(logits) -> repetition penalty over each beam's whole sequence
          (fake prefix included, Q4; on log-probs, so x*penalty) -> min_new_tokens mask;
          beam_sample then applies the warpers (min_keep 2) before the running beam score is added;
        * beam_search starts beams 1..K-1 at -1e9 (only beam 0 expands at the first step),
          beam_sample starts every beam at 0 (identical first-step rows: duplicate beams possible);
        * 2K candidates per utterance over the [K x V] scores: top-k (search) or multinomial without
          replacement from softmax(scores) sorted by score (sample); an eos candidate ranked < K closes a
          hypothesis (score / generated_len ** length_penalty, generated_len counting the eos slot),
          the first K non-eos candidates become the new beams;
        * an utterance is done once it holds K hypotheses and its worst one >= best candidate score /
          generated_len ** length_penalty; at max length the open beams are added as hypotheses.
        -> codes [B, n]: the best hypothesis per utterance, then the stop token (eos), padded with it.

        Test conveniences (no effect on the semantics): ``copies`` decodes every utterance ``copies`` times
        as independent utterances (b * copies + i; the prompt is prefilled once -- a row's prefill does not
        depend on the other rows -- for sampling statistics); ``trace`` (a list) receives one entry per step
        after its selection: the beams' sequences [R] and scores [B, K] and the step's 2K candidate scores
        [B, 2K] (ranked as the selection saw them; their K-th vs K+1-th gap is the step's tie margin).
        """
        emb, mask = self.prepare_inputs(conds, text_ids)
        B, s, D = emb.shape
        K = int(num_beams)
        sd = self.sd
        V = sd["mel_head.weight"].shape[0]
        stop = self.stop_mel
        start = sd["mel_embedding.weight"][self.start_mel] + sd["mel_pos_embedding.emb.weight"][0]
        x = torch.cat([emb, start.expand(B, 1, D)], 1)
        kv: List[Optional[tuple]] = [None] * self.L
        h = self.core(x, self._bias(mask, s + 1), kv)
        rows = torch.arange(B).repeat_interleave(K * copies)  # row b*K + k <- utterance b
        kv = [(k[rows], v[rows]) for k, v in kv]
        mask = mask[rows]
        logits = self.head(h[:, -1])[rows]
        B = B * copies
        R = B * K
        seen = torch.zeros(R, V, dtype=torch.bool)
        seen[:, 1] = True
        seen[:, self.start_mel] = True
        seqs = [[] for _ in range(R)]
        beam_scores = torch.zeros(B, K)
        if not do_sample:
            beam_scores[:, 1:] = -1e9
        hyps = [[] for _ in range(B)]  # list order matters for ties: (score, tokens)
        worst = [1e9] * B
        done = [False] * B

        def add(b, toks, score, glen):
            sc_ = score / (glen ** length_penalty)
            if len(hyps[b]) < K or sc_ > worst[b]:
                hyps[b].append((sc_, list(toks)))
                if len(hyps[b]) > K:
                    order = sorted((hs, i) for i, (hs, _) in enumerate(hyps[b]))
                    del hyps[b][order[0][1]]
                    worst[b] = order[1][0]
                else:
                    worst[b] = min(sc_, worst[b])

        for step in range(max_new_tokens):
            lp = torch.log_softmax(logits, -1)
            sc = self.penalize(lp, seen, repetition_penalty)
            if step < min_new_tokens:
                sc[:, stop] = float("-inf")
            if do_sample:
                sc = self.warp(sc, temperature, top_k, top_p, 2)
            sc = (sc + beam_scores.reshape(R, 1)).reshape(B, K * V)
            if do_sample:
                idx = torch.multinomial(torch.softmax(sc, -1), 2 * K, generator=generator)
                vals = torch.gather(sc, 1, idx)
                vals, order = torch.sort(vals, descending=True, dim=1)
                idx = torch.gather(idx, 1, order)
            else:
                vals, idx = torch.topk(sc, 2 * K, dim=1)
            glen = step + 1
            parent = torch.zeros(R, dtype=torch.long)
            token = torch.full((R,), stop, dtype=torch.long)
            new_scores = torch.zeros(B, K)
            for b in range(B):
                if done[b]:
                    parent[b * K:(b + 1) * K] = torch.arange(b * K, (b + 1) * K)
                    continue
                j = 0
                for rank in range(2 * K):
                    t, p, v = int(idx[b, rank] % V), int(idx[b, rank] // V), float(vals[b, rank])
                    if t == stop:
                        if rank >= K:
                            continue
                        add(b, seqs[b * K + p], v, glen)
                    else:
                        new_scores[b, j], token[b * K + j], parent[b * K + j] = v, t, b * K + p
                        j += 1
                    if j == K:
                        break
                if len(hyps[b]) >= K and worst[b] >= float(vals[b].max()) / (glen ** length_penalty):
                    done[b] = True
            if all(done):
                break
            # reorder the beams (HF _reorder_cache / input_ids[beam_idx]) and append the new tokens
            kv = [(k[parent], v[parent]) for k, v in kv]
            seen = seen[parent]
            seqs = [seqs[int(parent[r])] + [int(token[r])] for r in range(R)]
            seen[torch.arange(R), token] = True
            beam_scores = new_scores
            if trace is not None:
                trace.append({"seqs": [list(q) for q in seqs], "scores": beam_scores.clone(), "vals": vals.clone(),
                              "done": list(done)})
            if step == max_new_tokens - 1:
                break
            mask = torch.cat([mask, torch.ones(R, 1, dtype=mask.dtype)], 1)
            pos = mask.shape[1] - s  # quirk Q1
            e = sd["mel_embedding.weight"][token] + sd["mel_pos_embedding.emb.weight"][pos]
            h = self.core(e[:, None], self._bias(mask, 1), kv, self.sd_dec)
            logits = self.head(h[:, -1], self.sd_dec)
        for b in range(B):  # finalize
            if done[b]:
                continue
            for k in range(K):
                add(b, seqs[b * K + k], float(beam_scores[b, k]), len(seqs[b * K + k]))
        best = []
        for b in range(B):
            srt = sorted(hyps[b], key=lambda t: t[0])
            best.append(srt[-1][1])
        n = min(max(len(t) for t in best) + 1, max_new_tokens)
        out = torch.full((B, n), stop, dtype=torch.long)
        for b, t in enumerate(best):
            out[b, :len(t)] = torch.tensor(t, dtype=torch.long)
        return out

    def forced_logits(self, conds, text_ids, codes: torch.Tensor):
        """Teacher-forced decode: the logits (after penalty) the generate loop sees at each step when
        fed ``codes`` -> [B, n, V]. Lets fixtures compare per-step logits without free-running drift.
        (With ``sd_decode``: the prompt block through ``sd``, the fed codes through ``sd_decode`` over the
        prompt's KV cache -- one causal chunk, the same values as one step at a time.)"""
        emb, mask = self.prepare_inputs(conds, text_ids)
        B, s, D = emb.shape
        sd = self.sd
        start = sd["mel_embedding.weight"][self.start_mel] + sd["mel_pos_embedding.emb.weight"][0]
        x = torch.cat([emb, start.expand(B, 1, D)], 1)
        n = codes.shape[1]
        pos = torch.tensor([0] + list(range(2, n + 1)))  # positions 0, 2, 3, ... (Q1)
        tok = codes[:, : n - 1]
        e = sd["mel_embedding.weight"][tok] + sd["mel_pos_embedding.emb.weight"][pos[1:n]][None]
        mask_full = torch.cat([mask, torch.ones(B, n - 1, dtype=mask.dtype)], 1)
        if self.sd_dec is self.sd:
            full = torch.cat([x, e], 1)
            h = self.core(full, self._bias(mask_full, full.shape[1]))
            return self.head(h[:, s:])
        kv: List[Optional[tuple]] = [None] * self.L
        h0 = self.core(x, self._bias(mask, s + 1), kv)[:, -1:]
        out = [self.head(h0)]
        if n > 1:
            h1 = self.core(e, self._bias(mask_full, n - 1), kv, self.sd_dec)
            out.append(self.head(h1, self.sd_dec))
        return torch.cat(out, 1)

    # ---------------- post-processing + latent pass ----------------
    @staticmethod
    def remove_long_silence(codes: torch.Tensor, stop_mel: int = 8193, silent_token: int = 52, max_consecutive: int = 30):
        lens, rows, fixed = [], [], False
        for i in range(codes.shape[0]):
            c = codes[i]
            hits = (c == stop_mel).nonzero()
            n = int(hits[0]) if len(hits) else c.numel()
            if int((c == silent_token).sum()) > max_consecutive:
                keep, run = [], 0
                for k in range(n):
                    if int(c[k]) != silent_token:
                        keep.append(k)
                        run = 0
                    elif run < 10:
                        keep.append(k)
                        run += 1
                rows.append(c[keep])
                n = len(keep)
                fixed = True
            else:
                rows.append(c[:n])
            lens.append(n)
        if fixed:
            codes = torch.nn.utils.rnn.pad_sequence(rows, batch_first=True, padding_value=stop_mel) if len(rows) > 1 \
                else rows[0][None]
        m = max(lens)
        return codes[:, :m], torch.tensor(lens, dtype=torch.long)

    def latent(self, conds, text_ids, codes):
        """``UnifiedVoice.forward(..., return_latent=True)`` for ONE utterance (B=1, no padding).

        conds [1, 32, D]; text_ids [1, L] (as given; no 0/1 stripping on this path);
        codes [1, n] -> latent [1, n, D]."""
        sd = self.sd
        t = torch.cat([torch.tensor([[self.start_text]]), text_ids.long(), torch.tensor([[self.stop_text]])], 1)
        # gpt/model.py:559-566: text padded with stop (already full length), mel padded with stop
        m = torch.cat([torch.tensor([[self.start_mel]]), codes.long(), torch.tensor([[self.stop_mel]])], 1)
        # set_mel_padding: code_lens*1024 -> ceil(.)+1 >= n, so no in-range position is replaced
        te = sd["text_embedding.weight"][t] + sd["text_pos_embedding.emb.weight"][: t.shape[1]][None]
        me = sd["mel_embedding.weight"][m] + sd["mel_pos_embedding.emb.weight"][: m.shape[1]][None]
        x = torch.cat([conds.float(), te, me], 1)
        T = x.shape[1]
        h = self.core(x, self._bias(torch.ones(1, T), T))
        h = F.layer_norm(h[:, conds.shape[1]:], (self.D,), sd["final_norm.weight"], sd["final_norm.bias"], 1e-5)
        return h[:, -m.shape[1]:][:, :-2]
