"""Vocoder-only timing at the C3 shape (32 utterances x 400 latent frames, full IndexTTS-1.5 BigVGAN, seeded
weights): median of 5 HipBigVGAN.forward calls (one itts_bigvgan_forward each) after 2 warm-ups, HIP events.
Prints `<label> <ms>`; label from argv[1] (library / env variant)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "index-tts-dubbing_amd"))
from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import bigvgan_state_dict  # noqa: E402
from indextts.vocoder.bigvgan import HipBigVGAN  # noqa: E402


def main():
    cfg = load_config(default_config_path())
    voc = HipBigVGAN(bigvgan_state_dict(cfg.bigvgan, 0), cfg.bigvgan, "cuda")
    g = torch.Generator().manual_seed(0)
    lat = (torch.randn(32, 400, 1024, generator=g) * 0.5).to(torch.bfloat16).cuda()
    spk = torch.randn(32, 512, generator=g).cuda()
    lens = torch.full((32,), 400, dtype=torch.int32)
    ts = []
    for i in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        voc.forward(lat, lens, spk)
        b.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(a.elapsed_time(b))
    print(sys.argv[1] if len(sys.argv) > 1 else "default", round(sorted(ts)[2], 3), flush=True)


if __name__ == "__main__":
    main()
