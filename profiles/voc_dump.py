"""Dump the vocoder's PCM for a fixed synthetic batch (bit-identity A/B between two library builds:
ITTS_HIP_LIB selects the build).  usage: python profiles/voc_dump.py OUT.npy"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import numpy as np
import torch
from indextts.utils.config import default_config_path, load_config
from indextts.utils.synthetic import bigvgan_state_dict
from indextts.vocoder.bigvgan import HipBigVGAN

cfg = load_config(default_config_path())
voc = HipBigVGAN(bigvgan_state_dict(cfg.bigvgan, 0), cfg.bigvgan, "cuda")
g = torch.Generator().manual_seed(7)
B, T = 6, 160
lat = torch.randn(B, T, 1024, generator=g).to("cuda", torch.bfloat16)
spk = torch.randn(B, 512, generator=g).cuda()
lens = torch.tensor([160, 157, 99, 64, 31, 5], dtype=torch.int32)
wav, pcm = voc.forward(lat, lens, spk)
torch.cuda.synchronize()
np.save(sys.argv[1], pcm.cpu().numpy())
w = wav.float().cpu().numpy()
print("dumped", pcm.shape, float(np.abs(w).mean()))
