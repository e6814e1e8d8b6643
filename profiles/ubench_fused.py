"""(Historical: needs commit a0a8361; its multi-role launches were removed afterwards.)  Per-layer timing of the
fused decode launches (gpt_step.hip at that commit) against the per-kernel path they
replace, at the C3 shape (B = 32 rows, KV length ~283, IndexTTS-1.5 weights, all 20 layers' distinct
weights / caches so the bytes come from HBM as in the real step).  Graph-captured chains of 20
layers, HIP events, us per layer.  ITTS_HIP_LIB selects a timing build (ITTS_STEP_DIAG) of the
library: 1 = consumers skip their waits, 2 = consumer roles only, 3 = producer roles only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch  # noqa: E402

from indextts import _hip  # noqa: E402
from indextts.gpt.engine import HipGPT  # noqa: E402
from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import gpt_state_dict  # noqa: E402


def graph_us(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    tag = os.environ.get("UB_TAG", "product")
    cfg = load_config(default_config_path())
    eng = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.08), cfg.gpt, "cuda", dtype="bf16")
    lib, D, H, L = eng.lib, eng.D, eng.H, eng.L
    B, S = 32, 283
    st = eng._alloc_state(B, 400)
    st["s"] = S - 1 - 100
    st["t"].copy_(torch.tensor([100, 0, 0, 0], dtype=torch.int32))
    st["kc"].normal_()
    st["vc"].normal_()
    st["h"].copy_(torch.randn_like(st["h"].float()).to(st["h"].dtype))
    st["x"].normal_()
    eng._c_state(st)
    sync = st["sync"]
    wpl = (H + 8 + D // 32 + 3) // 4 * 4
    stream = _hip.stream_ptr
    qkv = st["qkv"][: B * 3 * D].view(B, 3 * D)
    kb, cbs, chs = S - 100, st["kc"].stride(1), st["kc"].stride(2)

    def f1_fused():
        sync.zero_()
        for li, ly in enumerate(eng.layers):
            _hip.check(lib.itts_decode_qkv_attn(
                st["h"].data_ptr(), D, ly.wx["qkv"]["w16"].data_ptr(), ly.wx["qkv"]["u"].data_ptr(),
                ly.wx["qkv"]["c"].data_ptr(), 1e-5, qkv.data_ptr(), 3 * D, st["kc"][li].data_ptr(),
                st["vc"][li].data_ptr(), cbs, chs, eng.max_kv, st["pad"].data_ptr(), kb, st["t"].data_ptr(),
                st["o"].data_ptr(), D, B, H, None, 0, sync[li * wpl:].data_ptr(), sync[-4:].data_ptr(), stream()), "f1")

    def f1_split():
        for li, ly in enumerate(eng.layers):
            eng._dgx(st["h"], ly.wx["qkv"], B, qkv, nwaves=4)
            kc, vc = st["kc"][li], st["vc"][li]
            _hip.check(lib.itts_attn_decode(qkv.data_ptr(), 3 * D, 1, B * 3 * D, None, kc.data_ptr(), vc.data_ptr(),
                                            kc.stride(0), kc.stride(1), eng.max_kv, st["pad"].data_ptr(), kb,
                                            st["t"].data_ptr(), st["o"].data_ptr(), D, B, H, 1, 1, stream()), "attn")

    def c_attn_only():
        for li, ly in enumerate(eng.layers):
            eng._dgx(st["h"], ly.wx["qkv"], B, qkv, nwaves=4)

    def f2_fused():
        sync.zero_()
        for li, ly in enumerate(eng.layers):
            _hip.check(lib.itts_decode_mlp(
                st["h"].data_ptr(), D, ly.wx["fc"]["w16"].data_ptr(), ly.wx["fc"]["u"].data_ptr(),
                ly.wx["fc"]["c"].data_ptr(), 1e-5, st["f"].data_ptr(), 4 * D, ly.w["proj"]["sk"].data_ptr(),
                ly.b["proj"].data_ptr(), st["ws"].data_ptr(), st["x"].data_ptr(), D, B, D, 8,
                sync[li * wpl + H:].data_ptr(), sync[-4:].data_ptr(), stream()), "f2")

    def f2_split():
        for li, ly in enumerate(eng.layers):
            eng._dgx(st["h"], ly.wx["fc"], B, st["f"], gelu=True)
            eng._dg(st["f"], ly.w["proj"], B, None, st["ws"], epi=2, ksplit=8)
            eng._reduce(st, 8, ly.b["proj"], (None, None))

    def attn_chain(hot):
        def f():
            for li in range(L):
                kc, vc = st["kc"][0 if hot else li], st["vc"][0 if hot else li]
                _hip.check(lib.itts_attn_decode(qkv.data_ptr(), 3 * D, 1, B * 3 * D, None, kc.data_ptr(),
                                                vc.data_ptr(), kc.stride(0), kc.stride(1), eng.max_kv,
                                                st["pad"].data_ptr(), kb, st["t"].data_ptr(), st["o"].data_ptr(), D,
                                                B, H, 1, 1, stream()), "attn")
        return f

    def c_proj():
        for li, ly in enumerate(eng.layers):
            eng._dgx(st["o"], ly.wx["o"], B, st["x"], epi=1, xh=st["h"])

    res = {}
    for name, fn in (("F1 fused", f1_fused), ("c_attn+attn", f1_split), ("c_attn", c_attn_only),
                     ("F2 fused", f2_fused), ("c_fc+proj+reduce", f2_split), ("attn.c_proj", c_proj),
                     ("attn cold KV", attn_chain(False)), ("attn hot KV", attn_chain(True))):
        res[name] = graph_us(fn) / L
    for k, v in res.items():
        print(f"[{tag}] {k:18s} {v:7.2f} us/layer", flush=True)


if __name__ == "__main__":
    main()
