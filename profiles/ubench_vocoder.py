"""Per-conv timings of the BigVGAN2 vocoder at C3 (B=32 x 400 frames): each igemm / amp_conv / act
launch timed with HIP events (eager, one forward), grouped by (kernel, C, taps)."""
import os, sys, collections
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch
from indextts.utils.config import default_config_path, load_config
from indextts.utils.synthetic import bigvgan_state_dict
from indextts.vocoder.bigvgan import HipBigVGAN

cfg = load_config(default_config_path())
voc = HipBigVGAN(bigvgan_state_dict(cfg.bigvgan, 0), cfg.bigvgan, "cuda")
B, T = 32, 400
g = torch.Generator().manual_seed(0)
lat = torch.randn(B, T, 1024, generator=g).to("cuda", torch.bfloat16)
spk = torch.randn(B, 512, generator=g).cuda()
lens = torch.full((B,), T, dtype=torch.int32)
# whole generator as one C call (the product path), then per-launch timings through the Python
# launch sequence (same kernels)
for it in range(3):
    torch.cuda.synchronize()
    c0 = torch.cuda.Event(enable_timing=True); c1 = torch.cuda.Event(enable_timing=True)
    c0.record()
    voc.forward(lat, lens, spk)
    c1.record()
    torch.cuda.synchronize()
print(f"vocoder forward (C call): {c0.elapsed_time(c1):.1f} ms")
voc.cforward = False
stats = collections.defaultdict(lambda: [0, 0.0, 0.0])
events = []
for name in ("_conv", "_amp", "_act"):
    orig = getattr(voc, name)
    def wrap(*a, _orig=orig, _name=name, **k):
        x = a[1]
        c = a[0]
        if _name == "_act":
            key = ("act", x.shape[2], 0)
            flops = 0.0
        else:
            key = (_name[1:], c.cin, c.ntaps)
            flops = 2.0 * voc.rows * c.cin * c.cout * c.ntaps
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = _orig(*a, **k)
        e1.record()
        events.append((key, e0, e1, flops, x.numel() * 2))
        return r
    setattr(voc, name, wrap)
for it in range(3):
    events.clear()
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    voc.forward(lat, lens, spk)
    t1.record()
    torch.cuda.synchronize()
tot = t0.elapsed_time(t1)
for key, e0, e1, fl, nb in events:
    s = stats[key]
    s[0] += 1; s[1] += e0.elapsed_time(e1); s[2] += fl
print(f"vocoder forward: {tot:.1f} ms; sum of timed launches {sum(v[1] for v in stats.values()):.1f} ms")
for key, (n, ms, fl) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
    print(f"{str(key):22s} n={n:3d} {ms:8.2f} ms  avg {ms / n * 1e3:8.1f} us  {fl / (ms * 1e-3) / 1e12 if fl else 0:7.1f} TF/s")
