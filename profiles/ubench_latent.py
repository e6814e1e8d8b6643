"""Per-launch timings of the teacher-forced latent pass at C3 (32 utterances: 32 cond + 50 text + 402 mel
positions each): HIP events around every GEMM / LayerNorm / attention launch of HipGPT._forward_rows."""
import collections
import os
import sys
import time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import numpy as np
import torch
from indextts import _hip
from indextts.gpt.engine import HipGPT
from indextts.utils.config import default_config_path, load_config
from indextts.utils.synthetic import gpt_state_dict

cfg = load_config(default_config_path())
eng = HipGPT(gpt_state_dict(cfg.gpt, seed=0, mel_head_std=0.08), cfg.gpt, "cuda", "bf16", max_kv=600)
eng.cseq = False  # per-launch timing needs the Python launch sequence (same kernels as the C call)
B = 32
g = np.random.default_rng(0)
conds = torch.from_numpy(g.normal(0, 1, (B, 32, 1024)).astype(np.float32)).cuda()
texts = [torch.from_numpy(g.integers(2, 12000, 48)).cuda() for _ in range(B)]
codes = [torch.from_numpy(g.integers(0, 8192, 400)).cuda() for _ in range(B)]
stats = collections.defaultdict(lambda: [0, 0.0])
events = []
for name in ("_gemm", "_ln"):
    orig = getattr(eng, name)
    def wrap(*a, _o=orig, _n=name, **k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = _o(*a, **k)
        e1.record()
        key = (_n, tuple(a[0].shape), a[1]["N"] if _n == "_gemm" else 0)
        events.append((key, e0, e1))
        return r
    setattr(eng, name, wrap)
for it in range(3):
    events.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.latent(conds, texts, codes)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
for key, e0, e1 in events:
    stats[key][0] += 1
    stats[key][1] += e0.elapsed_time(e1)
print(f"latent pass wall: {tot * 1e3:.1f} ms; timed launches {sum(v[1] for v in stats.values()):.1f} ms")
for key, (n, ms) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
    M = key[1][0]
    K = key[1][1]
    N = key[2]
    fl = 2.0 * M * N * K if key[0] == "_gemm" else 0
    print(f"{str(key):40s} n={n:3d} {ms:8.2f} ms avg {ms / n * 1e3:8.1f} us {fl * n / (ms * 1e-3) / 1e12 if fl else 0:7.1f} TF/s")
