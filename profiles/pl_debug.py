"""Phase-by-phase comparison of ONE persistent decode layer (gpt_layer.hip) with the launch chain
(gpt_step.hip) on layer 0 of the full IndexTTS-1.5 GPT: after a prefill, both paths run one decode
step over a 1-layer view of the weights (mode 2: logits only, no advance) from the same saved state;
the chain's q|k|v, attention output, c_fc output, mlp.c_proj partials, x / x^ and logits are compared
with the persistent layer's scratch regions (granules, o tiles, f tiles, partials)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "index-tts-dubbing_amd"))
os.environ["ITTS_PL"] = "1"
from indextts import _hip  # noqa: E402
from indextts.gpt.engine import HipGPT  # noqa: E402
from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import gpt_state_dict  # noqa: E402



def offsets(nbytes):
    """scratch regions of gpt_layer.hip, counted back from its end: err 256 B, trace 64 KiB, then P2, FC,
    XC, P1, OB, GQ (their sizes are fixed by the 128-row capacity)"""
    p2 = nbytes - 256 - 256 * 32 * 8 - 8 * 128 * 1024 * 4
    fc = p2 - 8 * 128 * 512 * 2
    xc = fc - 8 * 128 * 1024 * 2
    p1 = xc - 8 * 128 * 1024 * 4
    ob = p1 - 8 * 128 * 128 * 2
    gq = ob - 128 * 16 * 192 * 8
    return gq, ob, p1, xc, fc, p2


def cmp(name, a, b):
    a, b = a.float().cpu(), b.float().cpu()
    d = (a - b).abs()
    nz = int((a != b).sum())
    print(f"  {name:10s} shape={tuple(a.shape)} differ={nz} max|d|={float(d.max()):.3e} "
          f"max|ref|={float(b.abs().max()):.3e}", flush=True)
    if nz:
        idx = (a != b).nonzero()[:4].tolist()
        print(f"    first diffs at {idx}: pl={[float(a[tuple(i)]) for i in idx]} chain={[float(b[tuple(i)]) for i in idx]}")


def main(B):
    cfg = load_config(default_config_path())
    eng = _cache.get("eng")
    if eng is None:
        eng = _cache["eng"] = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.08), cfg.gpt, "cuda", dtype="bf16", max_kv=256)
    g = torch.Generator().manual_seed(5 + B)
    text = torch.randint(2, 12000, (B, 24), generator=g).cuda()
    conds = torch.randn(B, 32, 1024, generator=g).cuda()
    eng.pl = False
    for k in list(eng._lanes):
        del eng._lanes[k]
    eng.generate(conds, text, 1, use_graph=False)
    ln = [v for k, v in eng._lanes.items() if isinstance(k, tuple) and len(k) == 2 and k[0] == 0][0]
    st = ln["st"]
    torch.cuda.synchronize()
    keep = {k: st[k].clone() for k in ("x", "h", "t", "kc", "vc")}
    w1 = _hip.GptWeights.from_buffer_copy(eng._cweights)
    w1.n_layer = 1
    mode = _hip.Sampling(2, 0, 1.0, 1.0, 0, 1.0)
    cst = eng._c_state(st)
    lib = eng.lib
    s = _hip.stream_ptr()
    D = 1024
    print(f"B={B} kv_base={cst.kv_base} t={st['t'].tolist()}", flush=True)
    _hip.check(lib.itts_gpt_decode_step(ctypes.byref(w1), ctypes.byref(cst), ctypes.byref(mode), s), "chain")
    torch.cuda.synchronize()
    ch = {k: st[k].clone() for k in ("qkv", "o", "f", "ws", "x", "h", "logits")}
    for k, v in keep.items():
        st[k].copy_(v)
    eng._pl_scratch.zero_()
    _hip.check(lib.itts_gpt_decode_steps_pl(ctypes.byref(w1), eng._plw, eng._pl_scratch.data_ptr(), ctypes.byref(cst),
                                            ctypes.byref(mode), 1, s), "pl")
    torch.cuda.synchronize()
    print(f"  pl_error={eng.pl_error()}", flush=True)
    sc = eng._pl_scratch.view(torch.uint8)
    OFF_GQ, OFF_OB, OFF_P1, OFF_XC, OFF_FC, OFF_P2 = offsets(int(lib.itts_gpt_pl_scratch_bytes()))
    gq = sc[OFF_GQ:OFF_GQ + 128 * 16 * 192 * 8].view(torch.int64).view(128, 16, 192)[:B]
    gval = (gq & 0xFFFFFFFF).to(torch.int32).view(torch.float32)
    gtag = (gq >> 32)
    print(f"  granule tags: min={int(gtag.min())} max={int(gtag.max())}")
    # chain q|k|v [B][3D]: head h's [q | k | v] columns
    qkv = ch["qkv"].view(-1)[: B * 3 * D].view(B, 3, 16, 64).permute(0, 2, 1, 3).reshape(B, 16, 192)
    cmp("q|k|v", gval, qkv)
    ob = sc[OFF_OB:OFF_OB + 8 * 128 * 128 * 2].view(torch.bfloat16).view(8, 128, 2, 64)[:, :B]
    o_pl = ob.permute(1, 0, 2, 3).reshape(B, D)
    cmp("attn o", o_pl, ch["o"].view(-1)[: B * D].view(B, D))
    fcb = sc[OFF_FC:OFF_FC + 8 * 128 * 512 * 2].view(torch.bfloat16).view(8, 128, 512)[:, :B]
    f_pl = fcb.permute(1, 0, 2).reshape(B, 4 * D)
    cmp("c_fc f", f_pl, ch["f"].view(-1)[: B * 4 * D].view(B, 4 * D))
    p2 = sc[OFF_P2:OFF_P2 + 8 * 128 * 1024 * 4].view(torch.float32).view(8, 128, D)[:, :B]
    cmp("mlp part", p2, ch["ws"].view(-1)[: 8 * B * D].view(8, B, D))
    cmp("x", st["x"][:B], ch["x"][:B])
    cmp("x^", st["h"][:B], ch["h"][:B])
    cmp("logits", st["logits"][:B, :8194], ch["logits"][:B, :8194])


_cache = {}
if __name__ == "__main__":
    for B in [int(v) for v in (sys.argv[1:] or ["32", "1"])]:
        main(B)
