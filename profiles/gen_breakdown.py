"""Where the C3 generate() wall time goes besides the 400 graph replays: host wall per phase of one
greedy generate call (B = 32, L = 48, 400 codes, EOS suppressed), device synchronised at each mark."""
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
conds, _ = tts.prompt_features(mels, None)
ids = torch.full((B, L), tts.stop_text, dtype=torch.long)
for b, t in enumerate(texts):
    ids[b, : t.numel()] = t.reshape(-1).long()
ids = ids.to(dev)
gpt = tts.gpt
marks = {}
def wrap(name):
    orig = getattr(gpt, name)
    def f(*a, **k):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        r = orig(*a, **k)
        torch.cuda.synchronize(); marks[name] = marks.get(name, 0.0) + time.perf_counter() - t0
        return r
    setattr(gpt, name, f)
for n in ("prepare_inputs", "_start_lane"):
    wrap(n)
for rep in range(3):
    marks.clear()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    gpt.generate(conds, ids, N, repetition_penalty=10.0, min_new_tokens=N)
    torch.cuda.synchronize(); tot = time.perf_counter() - t0
    print(f"generate {tot * 1e3:.1f} ms; " + ", ".join(f"{k} {v * 1e3:.1f} ms" for k, v in marks.items()), flush=True)
