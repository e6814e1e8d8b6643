"""Per-layer timing of decode MLP launch variants at the C3 shape (B = 32 rows, IndexTTS-1.5, all 20
layers' distinct weights so the bytes come from HBM): graph-captured 20-layer chains, HIP events.
  split8:  c_fc (ln_2 folded, gelu) -> mlp.c_proj split-K 8 partials -> residual reduce   (product)
  fullk16: c_fc -> mlp.c_proj full K, 16 waves, residual epilogue (x += ., x^ = bf16 x)
  fullk8:  c_fc -> mlp.c_proj full K, 8 waves, residual epilogue
  c_fc / proj-only / reduce-only / c_attn / attn.c_proj: single launches for reference."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch  # noqa: E402

from indextts.gpt.engine import HipGPT  # noqa: E402
from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import gpt_state_dict  # noqa: E402
from ubench_fused import graph_us  # noqa: E402


def main():
    cfg = load_config(default_config_path())
    eng = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.08), cfg.gpt, "cuda", dtype="bf16")
    D, L = eng.D, eng.L
    B = 32
    st = eng._alloc_state(B, 400)
    st["h"].copy_(torch.randn_like(st["h"].float()).to(st["h"].dtype))
    st["x"].normal_()
    qkv = st["qkv"][: B * 3 * D].view(B, 3 * D)

    def chain(*parts):
        def f():
            for ly in eng.layers:
                for p in parts:
                    p(ly)
        return f

    c_fc = lambda ly: eng._dgx(st["h"], ly.wx["fc"], B, st["f"], gelu=True)  # noqa: E731
    proj8 = lambda ly: eng._dg(st["f"], ly.w["proj"], B, None, st["ws"], epi=2, ksplit=8)  # noqa: E731
    red = lambda ly: eng._reduce(st, 8, ly.b["proj"], (None, None))  # noqa: E731
    full16 = lambda ly: eng._dgx(st["f"], ly.wx["proj"], B, st["x"], epi=1, xh=st["h"], nwaves=16)  # noqa: E731
    full8 = lambda ly: eng._dgx(st["f"], ly.wx["proj"], B, st["x"], epi=1, xh=st["h"], nwaves=8)  # noqa: E731
    c_attn = lambda ly: eng._dgx(st["h"], ly.wx["qkv"], B, qkv)  # noqa: E731
    c_fc16 = lambda ly: eng._dgx(st["h"], ly.wx["fc"], B, st["f"], gelu=True, nwaves=16)  # noqa: E731
    c_attn16 = lambda ly: eng._dgx(st["h"], ly.wx["qkv"], B, qkv, nwaves=16)  # noqa: E731
    c_proj = lambda ly: eng._dgx(st["o"], ly.wx["o"], B, st["x"], epi=1, xh=st["h"])  # noqa: E731
    for name, fn in (("split8 (c_fc+proj8+reduce)", chain(c_fc, proj8, red)), ("fullk16 (c_fc+proj)", chain(c_fc, full16)),
                     ("fullk8 (c_fc+proj)", chain(c_fc, full8)), ("c_fc", chain(c_fc)), ("proj split8", chain(proj8)),
                     ("reduce", chain(red)), ("proj fullk16", chain(full16)), ("proj fullk8", chain(full8)),
                     ("c_attn", chain(c_attn)), ("attn.c_proj", chain(c_proj)), ("c_fc nw16", chain(c_fc16)),
                     ("c_attn nw16", chain(c_attn16)), ("fullk16 w/ c_fc nw16", chain(c_fc16, full16))):
        print(f"{name:28s} {graph_us(fn) / L:7.2f} us/layer", flush=True)


if __name__ == "__main__":
    main()
