"""Vocoder time inside the C3 pipeline vs standalone on the same inputs: wraps HipBigVGAN.forward
with HIP events during tts.synthesize (after the decode), then replays the captured (latent, lens,
spk) alone.  Prints the latent shape, the lengths and both times."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch
from bench import make_inputs
from indextts.pipeline import BatchedTTS
from indextts.utils.config import default_config_path, load_config
from indextts.utils.synthetic import bigvgan_state_dict, gpt_state_dict

cfg = load_config(default_config_path())
dev = torch.device("cuda:0")
N, L, B = 400, 48, 32
tts = BatchedTTS(gpt_state_dict(cfg.gpt, seed=0, mel_head_std=0.08), bigvgan_state_dict(cfg.bigvgan, seed=0),
                 cfg, dev, "bf16", max_kv=32 + L + 2 + 1 + N + 8)
mels, texts = make_inputs(cfg, list(range(B)), L, 511)
mels = [m.to(dev) for m in mels]
voc = tts.vocoder
orig = voc.forward
seen = {}
def fwd(latent, lens, spk, want_pcm=True):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = orig(latent, lens, spk, want_pcm)
    e1.record()
    torch.cuda.synchronize()
    seen["args"] = (latent, lens, spk)
    seen.setdefault("ms", []).append(e0.elapsed_time(e1))
    return r
voc.forward = fwd
for rep in range(3):
    ph = {}
    tts.synthesize(mels, texts, max_mel_tokens=N, min_new_tokens=N, timings=ph)
    print("phases ms:", {k: round(v * 1e3, 1) for k, v in ph.items()}, "vocoder events ms:", round(seen["ms"][-1], 1),
          flush=True)
latent, lens, spk = seen["args"]
print("latent", tuple(latent.shape), latent.dtype, "lens min/max/sum", int(lens.min()), int(lens.max()), int(lens.sum()))
for rep in range(3):
    fwd(latent, lens, spk)
    print("standalone vocoder ms:", round(seen["ms"][-1], 1), flush=True)
lat2 = torch.randn(B, 400, latent.shape[2], device=dev).to(torch.bfloat16)
for rep in range(2):
    fwd(lat2, torch.full((B,), 400, dtype=torch.int32), spk)
    print("standalone vocoder, T = 400 ms:", round(seen["ms"][-1], 1), flush=True)
