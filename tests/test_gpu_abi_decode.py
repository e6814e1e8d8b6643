"""The decode step driven through the C ABI alone (no HipGPT): a host that only has the header's
structs and entry points -- as a cgo / JNI / plain-C caller would -- packs the weights, allocates the
state from ``itts_gpt_decode_state_bytes`` and calls ``itts_gpt_decode_step`` once per token.

Check: teacher-forced decoding of a mel-token sequence from an empty cache (kv_base = 0; the first
input is mel_emb[start] + mel_pos[0] as after the prefill, token j >= 1 enters as mel_emb[t_j] +
mel_pos[j + 2], quirk Q1) against an fp32 torch GPT-2 forward of the same sequence (HF
modeling_gpt2.py:246-306, ln_f + final_norm + mel_head, gpt/model.py:48,180).  bf16 weights and
activations: per-step logits relative RMS error <= 2e-2; the sampler's recorded argmax equals the
reference argmax wherever the reference top-1 / top-2 margin exceeds 0.1.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _t(v):
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))


def _reference_logits(sd, cfg, tokens, pos):
    """fp32 GPT-2 over inputs mel_emb[tokens] + mel_pos[pos] ([R, T]); logits [R, T, V]."""
    D, H = int(cfg.model_dim), int(cfg.heads)
    x = _t(sd["mel_embedding.weight"]).float()[tokens] + _t(sd["mel_pos_embedding.emb.weight"]).float()[pos]
    R, T, _ = x.shape
    mask = torch.full((T, T), float("-inf")).triu(1)
    for i in range(int(cfg.layers)):
        p = f"gpt.h.{i}."
        g = lambda k: _t(sd[p + k]).float()  # noqa: E731
        h = F.layer_norm(x, (D,), g("ln_1.weight"), g("ln_1.bias"), 1e-5)
        qkv = h @ g("attn.c_attn.weight") + g("attn.c_attn.bias")
        q, k, v = (t.view(R, T, H, 64).transpose(1, 2) for t in qkv.split(D, -1))
        a = torch.softmax(q @ k.transpose(-1, -2) / 8.0 + mask, -1) @ v
        x = x + a.transpose(1, 2).reshape(R, T, D) @ g("attn.c_proj.weight") + g("attn.c_proj.bias")
        h = F.layer_norm(x, (D,), g("ln_2.weight"), g("ln_2.bias"), 1e-5)
        f = F.gelu(h @ g("mlp.c_fc.weight") + g("mlp.c_fc.bias"), approximate="tanh")
        x = x + f @ g("mlp.c_proj.weight") + g("mlp.c_proj.bias")
    x = F.layer_norm(x, (D,), _t(sd["gpt.ln_f.weight"]).float(), _t(sd["gpt.ln_f.bias"]).float(), 1e-5)
    x = F.layer_norm(x, (D,), _t(sd["final_norm.weight"]).float(), _t(sd["final_norm.bias"]).float(), 1e-5)
    return x @ _t(sd["mel_head.weight"]).float().t() + _t(sd["mel_head.bias"]).float()


def test_decode_step_through_the_abi_only():
    from indextts import _hip
    from indextts.gpt.engine import fold_ln_weights, pack_skinny
    from indextts.utils.config import tiny_config
    from indextts.utils.synthetic import gpt_state_dict

    lib = _hip.load()
    cfg = tiny_config().gpt
    sd = gpt_state_dict(cfg, 0, 0.08)
    dev = "cuda"
    D, H, L, V = int(cfg.model_dim), int(cfg.heads), int(cfg.layers), int(cfg.number_mel_codes)
    Vp = (V + 15) // 16 * 16
    start, stop = int(cfg.start_mel_token), int(cfg.stop_mel_token)
    keep = []  # device tensors the structs point at

    def dev32(v):
        t = _t(v).float().contiguous().to(dev)
        keep.append(t)
        return t.data_ptr()

    def ln(i, n):
        return sd[f"gpt.h.{i}.ln_{n}.weight"], sd[f"gpt.h.{i}.ln_{n}.bias"]

    layers = (_hip.GptLayerW * L)()
    for i in range(L):
        p = f"gpt.h.{i}."
        qkv = fold_ln_weights(sd[p + "attn.c_attn.weight"], sd[p + "attn.c_attn.bias"], ln(i, 1), dev)
        o = fold_ln_weights(sd[p + "attn.c_proj.weight"], sd[p + "attn.c_proj.bias"], None, dev)
        fc = fold_ln_weights(sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"], ln(i, 2), dev)
        proj = pack_skinny(_t(sd[p + "mlp.c_proj.weight"]).float().t().contiguous()).to(dev)
        ow = pack_skinny(_t(sd[p + "attn.c_proj.weight"]).float().t().contiguous()).to(dev)  # 32-column, split-K
        keep.extend([qkv, o, fc, proj, ow])
        layers[i] = _hip.GptLayerW(qkv["w16"].data_ptr(), qkv["u"].data_ptr(), qkv["c"].data_ptr(),
                                   o["w16"].data_ptr(), o["c"].data_ptr(), fc["w16"].data_ptr(), fc["u"].data_ptr(),
                                   fc["c"].data_ptr(), proj.data_ptr(), dev32(sd[p + "mlp.c_proj.bias"]),
                                   ow.data_ptr())
    head = pack_skinny(_t(sd["mel_head.weight"]).float().contiguous()).to(dev)
    keep.append(head)
    w = _hip.GptWeights(L, D, H, V, Vp, start, stop, layers, dev32(sd["gpt.ln_f.weight"]),
                        dev32(sd["gpt.ln_f.bias"]), dev32(sd["final_norm.weight"]), dev32(sd["final_norm.bias"]),
                        head.data_ptr(), dev32(sd["mel_head.bias"]), dev32(sd["mel_embedding.weight"]),
                        dev32(sd["mel_pos_embedding.emb.weight"]))

    R, T, max_kv = 5, 24, 32
    sizes = (ctypes.c_int64 * _hip.GPT_STATE_NBUF)()
    assert lib.itts_gpt_decode_state_bytes(ctypes.byref(w), R, max_kv, T, sizes) == 0
    buf = [torch.zeros(int(n), dtype=torch.uint8, device=dev) for n in sizes]
    x, xh, qkv, o, f, part, logits, kc, vc, pad, tst, seen, done, codes = buf
    g = torch.Generator().manual_seed(3)
    tokens = torch.randint(0, 8192, (R, T), generator=g)
    tokens[:, 0] = start
    pos = torch.cat([torch.zeros(R, 1, dtype=torch.long), torch.arange(3, T + 2).expand(R, T - 1)], 1)
    forced = torch.full((R, T), stop, dtype=torch.int32)
    forced[:, 1:] = tokens[:, 1:].int()
    forced = forced.to(dev)
    # the first input (what the prefill leaves behind): x = mel_emb[start] + mel_pos[0], xh = bf16(x)
    x0 = (_t(sd["mel_embedding.weight"]).float()[start] + _t(sd["mel_pos_embedding.emb.weight"]).float()[0])
    x.view(torch.float32).view(R, D).copy_(x0.expand(R, D))
    xh.view(torch.bfloat16).view(-1, D)[:R].copy_(x0.expand(R, D).to(torch.bfloat16))
    st = _hip.GptDecodeState(R, max_kv, 0, T, x.data_ptr(), xh.data_ptr(), qkv.data_ptr(), o.data_ptr(),
                             f.data_ptr(), part.data_ptr(), logits.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                             pad.data_ptr(), tst.data_ptr(), None, 0, seen.data_ptr(), done.data_ptr(),
                             codes.data_ptr(), forced.data_ptr())
    smp = _hip.Sampling(0, T, 1.0, 1.0, 0, 1.0)  # greedy, no stop before T, penalty 1 (none)
    got = []
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(T - 1):
        _hip.check(lib.itts_gpt_decode_step(ctypes.byref(w), ctypes.byref(st), ctypes.byref(smp), stream),
                   "itts_gpt_decode_step")
        got.append(logits.view(torch.float32).view(R, Vp)[:, :V].clone())
    torch.cuda.synchronize()
    assert int(tst.view(torch.int32)[0]) == T - 1  # the device step counter advanced once per call
    got = torch.stack(got, 1).cpu()                                  # [R, T-1, V]
    ref = _reference_logits(sd, cfg, tokens[:, : T - 1], pos[:, : T - 1])
    rel = float(((got - ref).pow(2).mean() / ref.pow(2).mean()).sqrt())
    assert rel <= 2e-2, rel
    sel = ref.clone()
    sel[..., stop] = float("-inf")  # min_new_tokens = T suppresses the stop token
    top2 = sel.topk(2, -1).values
    margin = top2[..., 0] - top2[..., 1]
    chosen = codes.view(torch.int32).view(R, T).cpu()[:, 1:T].long()  # argmax recorded at col j + 1
    ok = (chosen == sel.argmax(-1)) | (margin <= 0.1)
    assert bool(ok.all()), (chosen, ref.argmax(-1))


@pytest.mark.parametrize("size", ["tiny", "full"])
def test_prefill_decode_latent_through_the_abi_only(size):
    """The whole GPT side of one infer() through the header's entry points alone -- itts_gpt_prefill
    (prompt block -> KV cache, head, first token), itts_gpt_decode_steps / itts_gpt_decode_step (the
    loop), itts_gpt_forward_rows (teacher-forced latent pass, gpt/model.py:521-578) -- over weights the
    test packs itself and state sized by itts_gpt_decode_state_bytes, on a left-padded batch; codes and
    latents bit-identical to HipGPT's Python launch sequence (ITTS_CSEQ=0 path)."""
    from indextts import _hip
    from indextts.gpt.engine import HipGPT, fold_ln_weights, pack_skinny
    from indextts.utils.config import default_config_path, load_config, tiny_config
    from indextts.utils.synthetic import gpt_state_dict
    from indextts.vocoder.bigvgan import pack_taps

    lib = _hip.load()
    cfg = (tiny_config() if size == "tiny" else load_config(default_config_path())).gpt
    sd = gpt_state_dict(cfg, 0, 0.08)
    dev = "cuda"
    D, H, L, V = int(cfg.model_dim), int(cfg.heads), int(cfg.layers), int(cfg.number_mel_codes)
    Vp = (V + 15) // 16 * 16
    start, stop = int(cfg.start_mel_token), int(cfg.stop_mel_token)
    B, N = 4, 40
    g = torch.Generator().manual_seed(5)
    conds = torch.randn(B, 32, D, generator=g).cuda()
    text = torch.randint(2, 6000, (B, 12), generator=g)
    text[0, :5] = 1  # left-padded rows (stop id stripped, Q3)
    text[2, :2] = 1
    text = text.cuda()

    # ---- reference: HipGPT with the Python launch sequences
    eng = HipGPT(sd, cfg, dev, dtype="bf16")
    eng.cseq = False
    want = eng.generate(conds, text, N, min_new_tokens=N, repetition_penalty=10.0).cpu()
    texts = [t[t != 1] for t in text]
    lat_want, lat_n = eng.latent(conds, texts, [c for c in want])
    emb, pad, s = eng.prepare_inputs(conds, text)  # host-side table lookups (prepare_gpt_inputs)
    torch.cuda.synchronize()
    del eng

    # ---- ABI only
    keep = []

    def dev32(v):
        t = _t(v).float().contiguous().to(dev)
        keep.append(t)
        return t.data_ptr()

    def lnp(i, n):
        return sd[f"gpt.h.{i}.ln_{n}.weight"], sd[f"gpt.h.{i}.ln_{n}.bias"]

    layers = (_hip.GptLayerW * L)()
    seq_layers = (_hip.GptSeqLayerW * L)()
    for i in range(L):
        p = f"gpt.h.{i}."
        qkv = fold_ln_weights(sd[p + "attn.c_attn.weight"], sd[p + "attn.c_attn.bias"], lnp(i, 1), dev)
        o = fold_ln_weights(sd[p + "attn.c_proj.weight"], sd[p + "attn.c_proj.bias"], None, dev)
        fc = fold_ln_weights(sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"], lnp(i, 2), dev)
        proj = pack_skinny(_t(sd[p + "mlp.c_proj.weight"]).float().t().contiguous()).to(dev)
        ow = pack_skinny(_t(sd[p + "attn.c_proj.weight"]).float().t().contiguous()).to(dev)  # 32-column, split-K
        keep.extend([qkv, o, fc, proj, ow])
        layers[i] = _hip.GptLayerW(qkv["w16"].data_ptr(), qkv["u"].data_ptr(), qkv["c"].data_ptr(),
                                   o["w16"].data_ptr(), o["c"].data_ptr(), fc["w16"].data_ptr(), fc["u"].data_ptr(),
                                   fc["c"].data_ptr(), proj.data_ptr(), dev32(sd[p + "mlp.c_proj.bias"]),
                                   ow.data_ptr())
        ig = []
        for k in ("attn.c_attn", "attn.c_proj", "mlp.c_fc", "mlp.c_proj"):
            wt = _t(sd[p + k + ".weight"]).float().t().contiguous()  # HF Conv1D [in, out] -> [out, in]
            t = pack_taps([wt], wt.shape[1], wt.shape[0]).to(dev)
            keep.append(t)
            ig.append(t.data_ptr())
        seq_layers[i] = _hip.GptSeqLayerW(*ig, *[dev32(sd[p + k + ".bias"]) for k in
                                                 ("attn.c_attn", "attn.c_proj", "mlp.c_fc", "mlp.c_proj")],
                                          dev32(lnp(i, 1)[0]), dev32(lnp(i, 1)[1]), dev32(lnp(i, 2)[0]),
                                          dev32(lnp(i, 2)[1]))
    head = pack_skinny(_t(sd["mel_head.weight"]).float().contiguous()).to(dev)
    keep.append(head)
    lnf = (dev32(sd["gpt.ln_f.weight"]), dev32(sd["gpt.ln_f.bias"]), dev32(sd["final_norm.weight"]),
           dev32(sd["final_norm.bias"]))
    w = _hip.GptWeights(L, D, H, V, Vp, start, stop, layers, *lnf, head.data_ptr(), dev32(sd["mel_head.bias"]),
                        dev32(sd["mel_embedding.weight"]), dev32(sd["mel_pos_embedding.emb.weight"]))
    ws = _hip.GptSeqWeights(L, D, H, _hip.BF16, seq_layers, *lnf, None)

    max_kv = s + 1 + N + 8
    sizes = (ctypes.c_int64 * _hip.GPT_STATE_NBUF)()
    assert lib.itts_gpt_decode_state_bytes(ctypes.byref(w), B, max_kv, N, sizes) == 0
    buf = [torch.zeros(int(n), dtype=torch.uint8, device=dev) for n in sizes]
    x, xh, qkv, o, f, part, logits, kc, vc, padb, tst, seen, done, codes = buf
    padb.view(torch.int32).copy_(pad)
    seen.view(B, Vp)[:, 1] = 1  # the prompt's fake ids 1 and 8192 count for the repetition penalty (Q4)
    seen.view(B, Vp)[:, start] = 1
    codes.view(torch.int32).fill_(stop)
    st = _hip.GptDecodeState(B, max_kv, s + 1, N, x.data_ptr(), xh.data_ptr(), qkv.data_ptr(), o.data_ptr(),
                             f.data_ptr(), part.data_ptr(), logits.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                             padb.data_ptr(), tst.data_ptr(), None, 0, seen.data_ptr(), done.data_ptr(),
                             codes.data_ptr(), None)
    smp = _hip.Sampling(0, N, 10.0, 1.0, 0, 1.0)
    stream = torch.cuda.current_stream().cuda_stream
    M = B * (s + 1)
    work = torch.empty(int(lib.itts_gpt_forward_rows_workspace_bytes(ctypes.byref(ws), M)), dtype=torch.uint8,
                       device=dev)
    xin = emb.reshape(M, D).contiguous()
    starts = (torch.arange(B, dtype=torch.int32) * (s + 1)).to(dev)
    lens = torch.full((B,), s + 1, dtype=torch.int32, device=dev)
    last = (starts + s).contiguous()
    _hip.check(lib.itts_gpt_prefill(ctypes.byref(ws), ctypes.byref(w), ctypes.byref(st), xin.data_ptr(), s,
                                    starts.data_ptr(), lens.data_ptr(), last.data_ptr(), ctypes.byref(smp),
                                    work.data_ptr(), stream), "itts_gpt_prefill")
    done_steps = 1
    while done_steps < N:  # 4 steps per call while they fit, then single steps
        n = 4 if done_steps + 4 <= N else 1
        if n > 1:
            _hip.check(lib.itts_gpt_decode_steps(ctypes.byref(w), ctypes.byref(st), ctypes.byref(smp), n, stream),
                       "itts_gpt_decode_steps")
        else:
            _hip.check(lib.itts_gpt_decode_step(ctypes.byref(w), ctypes.byref(st), ctypes.byref(smp), stream),
                       "itts_gpt_decode_step")
        done_steps += n
    torch.cuda.synchronize()
    got = codes.view(torch.int32).view(B, N).cpu().long()
    assert torch.equal(got[:, : want.shape[1]], want), (got, want)

    # teacher-forced latent pass: [conds ; text_emb + text_pos ; mel_emb + mel_pos] per row, packed
    te, tp = _t(sd["text_embedding.weight"]).float(), _t(sd["text_pos_embedding.emb.weight"]).float()
    me, mp = _t(sd["mel_embedding.weight"]).float(), _t(sd["mel_pos_embedding.emb.weight"]).float()
    rows, st_l, ln_l, idx = [], [], [], []
    off = 0
    for b in range(B):
        tt = torch.cat([torch.tensor([int(cfg.start_text_token)]), texts[b].cpu(), torch.tensor([int(cfg.stop_text_token)])])
        mm = torch.cat([torch.tensor([start]), want[b], torch.tensor([stop])])
        r = torch.cat([conds[b].cpu(), te[tt] + tp[torch.arange(tt.numel())], me[mm] + mp[torch.arange(mm.numel())]])
        rows.append(r)
        st_l.append(off)
        ln_l.append(r.shape[0])
        first = off + 32 + tt.numel()
        idx.append(torch.arange(first, first + int(lat_n[b])))
        off += r.shape[0]
    xl = torch.cat(rows).to(dev).contiguous()
    Tm = int(lat_n.max())
    out_idx = torch.zeros(B, Tm, dtype=torch.int32)
    for b in range(B):
        out_idx[b, : idx[b].numel()] = idx[b].int()
    out_idx = out_idx.to(dev).view(-1)
    lat = torch.empty(B, Tm, D, dtype=torch.bfloat16, device=dev)
    work = torch.empty(int(lib.itts_gpt_forward_rows_workspace_bytes(ctypes.byref(ws), xl.shape[0])),
                       dtype=torch.uint8, device=dev)
    s_t, l_t = torch.tensor(st_l, dtype=torch.int32, device=dev), torch.tensor(ln_l, dtype=torch.int32, device=dev)
    _hip.check(lib.itts_gpt_forward_rows(ctypes.byref(ws), xl.data_ptr(), xl.shape[0], s_t.data_ptr(), l_t.data_ptr(),
                                         None, B, max(ln_l), None, None, 0, 0, 0, _hip.BF16, out_idx.data_ptr(),
                                         B * Tm, lat.data_ptr(), _hip.BF16, work.data_ptr(), stream),
               "itts_gpt_forward_rows")
    torch.cuda.synchronize()
    for b in range(B):
        n = int(lat_n[b])
        assert torch.equal(lat[b, :n].cpu(), lat_want[b, :n].cpu()), b


def _abi_pack_layers(lib, sd, L, D, H, dev, keep):
    """ItTsGptLayerW / ItTsGptPlLayerW arrays built with the header's host packers only (itts_gpt_fold_ln,
    itts_gpt_pack_frag, itts_gpt_pack_qkv12), as a host without Python would: host buffers in, device
    copies out."""
    from indextts import _hip

    def host(v):
        return _t(v).detach().float().cpu().contiguous()

    def todev(t):
        d = t.to(dev)
        keep.append(d)
        return d.data_ptr()

    def fold(w_io, bias, ln):
        w, b = host(w_io), host(bias)
        K, N = w.shape
        wt = torch.empty(N, K, dtype=torch.bfloat16)
        u, c = torch.empty(N), torch.empty(N)
        g = None if ln is None else host(ln[0])
        bb = None if ln is None else host(ln[1])
        _hip.check(lib.itts_gpt_fold_ln(w.data_ptr(), b.data_ptr(), None if g is None else g.data_ptr(),
                                        None if bb is None else bb.data_ptr(), K, N, wt.data_ptr(),
                                        u.data_ptr(), c.data_ptr()), "itts_gpt_fold_ln")
        return wt, u, c

    def frag(wt, dtype, cols):
        N, K = wt.shape
        Np = (N + cols - 1) // cols * cols
        out = torch.empty(Np * K, dtype=torch.bfloat16)
        _hip.check(lib.itts_gpt_pack_frag(wt.data_ptr(), dtype, N, K, cols, out.data_ptr()), "itts_gpt_pack_frag")
        return out

    layers = (_hip.GptLayerW * L)()
    pls = (_hip.GptPlLayerW * L)()
    for i in range(L):
        p = f"gpt.h.{i}."
        ln1 = (sd[p + "ln_1.weight"], sd[p + "ln_1.bias"])
        ln2 = (sd[p + "ln_2.weight"], sd[p + "ln_2.bias"])
        q_wt, q_u, q_c = fold(sd[p + "attn.c_attn.weight"], sd[p + "attn.c_attn.bias"], ln1)
        o_wt, _, o_c = fold(sd[p + "attn.c_proj.weight"], sd[p + "attn.c_proj.bias"], None)
        f_wt, f_u, f_c = fold(sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"], ln2)
        proj_t = host(sd[p + "mlp.c_proj.weight"]).t().contiguous()
        w12 = torch.empty(256 * (D // 32) * 4 * 12 * 8, dtype=torch.bfloat16)
        uc = torch.empty(256 * 2 * 12)
        _hip.check(lib.itts_gpt_pack_qkv12(q_wt.data_ptr(), q_u.data_ptr(), q_c.data_ptr(), D, H, w12.data_ptr(),
                                           uc.data_ptr()), "itts_gpt_pack_qkv12")
        layers[i] = _hip.GptLayerW(todev(frag(q_wt, _hip.BF16, 16)), todev(q_u), todev(q_c),
                                   todev(frag(o_wt, _hip.BF16, 16)), todev(o_c), todev(frag(f_wt, _hip.BF16, 16)),
                                   todev(f_u), todev(f_c), todev(frag(proj_t, _hip.F32, 32)),
                                   todev(host(sd[p + "mlp.c_proj.bias"])), todev(frag(o_wt, _hip.BF16, 32)))
        pls[i] = _hip.GptPlLayerW(todev(w12), todev(uc))
    head = todev(frag(host(sd["mel_head.weight"]), _hip.F32, 32))
    return layers, pls, head


def test_persistent_decode_through_the_abi_only():
    """The default decode path (itts_gpt_decode_steps_pl: every layer one persistent launch) driven through
    the header alone -- weights packed by the host packers, the scratch sized by itts_gpt_pl_scratch_bytes and
    zero-filled, prefill by itts_gpt_prefill, 8 steps per call -- at the full IndexTTS-1.5 size on a
    left-padded batch: codes bit-identical to HipGPT's launch chain (ITTS_PL=0, Python launch sequences)."""
    import os
    from indextts import _hip
    from indextts.gpt.engine import HipGPT
    from indextts.utils.config import default_config_path, load_config
    from indextts.utils.synthetic import gpt_state_dict
    from indextts.vocoder.bigvgan import pack_taps

    lib = _hip.load()
    cfg = load_config(default_config_path()).gpt
    sd = gpt_state_dict(cfg, 0, 0.08)
    dev = "cuda"
    D, H, L, V = int(cfg.model_dim), int(cfg.heads), int(cfg.layers), int(cfg.number_mel_codes)
    Vp = (V + 15) // 16 * 16
    start, stop = int(cfg.start_mel_token), int(cfg.stop_mel_token)
    B, N = 6, 41
    g = torch.Generator().manual_seed(15)
    conds = torch.randn(B, 32, D, generator=g).cuda()
    text = torch.randint(2, 6000, (B, 20), generator=g)
    text[1, :7] = 1
    text[4, :3] = 1
    text = text.cuda()
    old = os.environ.get("ITTS_PL")
    os.environ["ITTS_PL"] = "0"
    try:
        eng = HipGPT(sd, cfg, dev, dtype="bf16")
    finally:
        if old is None:
            del os.environ["ITTS_PL"]
        else:
            os.environ["ITTS_PL"] = old
    eng.cseq = False
    want = eng.generate(conds, text, N, min_new_tokens=N, repetition_penalty=10.0).cpu()
    emb, pad, s = eng.prepare_inputs(conds, text)
    torch.cuda.synchronize()
    del eng
    torch.cuda.empty_cache()

    keep = []
    layers, pls, head = _abi_pack_layers(lib, sd, L, D, H, dev, keep)

    def dev32(v):
        t = _t(v).float().contiguous().to(dev)
        keep.append(t)
        return t.data_ptr()

    lnf = (dev32(sd["gpt.ln_f.weight"]), dev32(sd["gpt.ln_f.bias"]), dev32(sd["final_norm.weight"]),
           dev32(sd["final_norm.bias"]))
    w = _hip.GptWeights(L, D, H, V, Vp, start, stop, layers, *lnf, head, dev32(sd["mel_head.bias"]),
                        dev32(sd["mel_embedding.weight"]), dev32(sd["mel_pos_embedding.emb.weight"]))
    if not lib.itts_gpt_pl_supported(ctypes.byref(w), B):
        pytest.skip("persistent layer not available on this device")
    seq_layers = (_hip.GptSeqLayerW * L)()
    for i in range(L):
        p = f"gpt.h.{i}."
        ig = []
        for k in ("attn.c_attn", "attn.c_proj", "mlp.c_fc", "mlp.c_proj"):
            wt = _t(sd[p + k + ".weight"]).float().t().contiguous()
            t = pack_taps([wt], wt.shape[1], wt.shape[0]).to(dev)
            keep.append(t)
            ig.append(t.data_ptr())
        seq_layers[i] = _hip.GptSeqLayerW(*ig, *[dev32(sd[p + k + ".bias"]) for k in
                                                 ("attn.c_attn", "attn.c_proj", "mlp.c_fc", "mlp.c_proj")],
                                          dev32(sd[p + "ln_1.weight"]), dev32(sd[p + "ln_1.bias"]),
                                          dev32(sd[p + "ln_2.weight"]), dev32(sd[p + "ln_2.bias"]))
    ws = _hip.GptSeqWeights(L, D, H, _hip.BF16, seq_layers, *lnf, None)
    max_kv = s + 1 + N + 8
    sizes = (ctypes.c_int64 * _hip.GPT_STATE_NBUF)()
    assert lib.itts_gpt_decode_state_bytes(ctypes.byref(w), B, max_kv, N, sizes) == 0
    buf = [torch.zeros(int(n), dtype=torch.uint8, device=dev) for n in sizes]
    x, xh, qkv, o, f, part, logits, kc, vc, padb, tst, seen, done, codes = buf
    padb.view(torch.int32).copy_(pad)
    seen.view(B, Vp)[:, 1] = 1
    seen.view(B, Vp)[:, start] = 1
    codes.view(torch.int32).fill_(stop)
    st = _hip.GptDecodeState(B, max_kv, s + 1, N, x.data_ptr(), xh.data_ptr(), qkv.data_ptr(), o.data_ptr(),
                             f.data_ptr(), part.data_ptr(), logits.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                             padb.data_ptr(), tst.data_ptr(), None, 0, seen.data_ptr(), done.data_ptr(),
                             codes.data_ptr(), None)
    smp = _hip.Sampling(0, N, 10.0, 1.0, 0, 1.0)
    scratch = torch.zeros(int(lib.itts_gpt_pl_scratch_bytes()), dtype=torch.uint8, device=dev)
    assert scratch.data_ptr() % 256 == 0
    stream = torch.cuda.current_stream().cuda_stream
    M = B * (s + 1)
    work = torch.empty(int(lib.itts_gpt_forward_rows_workspace_bytes(ctypes.byref(ws), M)), dtype=torch.uint8,
                       device=dev)
    xin = emb.reshape(M, D).contiguous()
    starts = (torch.arange(B, dtype=torch.int32) * (s + 1)).to(dev)
    lens = torch.full((B,), s + 1, dtype=torch.int32, device=dev)
    _hip.check(lib.itts_gpt_prefill(ctypes.byref(ws), ctypes.byref(w), ctypes.byref(st), xin.data_ptr(), s,
                                    starts.data_ptr(), lens.data_ptr(), (starts + s).contiguous().data_ptr(),
                                    ctypes.byref(smp), work.data_ptr(), stream), "itts_gpt_prefill")
    done_steps = 1
    while done_steps < N:  # 8 steps per call while they fit, then single steps
        n = 8 if done_steps + 8 <= N else 1
        _hip.check(lib.itts_gpt_decode_steps_pl(ctypes.byref(w), pls, scratch.data_ptr(), ctypes.byref(st),
                                                ctypes.byref(smp), n, stream), "itts_gpt_decode_steps_pl")
        done_steps += n
    code = ctypes.c_int(-1)
    _hip.check(lib.itts_gpt_pl_error(scratch.data_ptr(), stream, ctypes.byref(code)), "itts_gpt_pl_error")
    assert code.value == 0
    got = codes.view(torch.int32).view(B, N).cpu().long()
    assert torch.equal(got[:, : want.shape[1]], want), (got, want)
