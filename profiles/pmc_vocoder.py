"""Workload for the rocprofv3 PMC passes (HBM traffic of the vocoder conv kernel).

Runs the BigVGAN2 forward of bench.py's C3 step (B=32 utterances x 400 latent frames, seeded random
latents/speaker embeddings, random-init IndexTTS-1.5 vocoder weights) twice; the second forward's
``igemm_kernel`` dispatches are the ones `profiles/traffic.py` averages.

    cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python profiles/pmc_vocoder.py
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python profiles/pmc_vocoder.py
    python profiles/traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/traffic_r01.json
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "index-tts-dubbing_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import bigvgan_state_dict  # noqa: E402
from indextts.vocoder.bigvgan import HipBigVGAN  # noqa: E402


def main():
    cfg = load_config(default_config_path())
    voc = HipBigVGAN(bigvgan_state_dict(cfg.bigvgan, 0), cfg.bigvgan, "cuda")
    g = torch.Generator().manual_seed(0)
    B, T = 32, 400
    lat = torch.randn(B, T, int(cfg.bigvgan.gpt_dim), generator=g).to("cuda", torch.bfloat16)
    spk = torch.randn(B, 512, generator=g).cuda()
    lens = torch.full((B,), T, dtype=torch.int32)
    for _ in range(2):
        voc.forward(lat, lens, spk)
    torch.cuda.synchronize()
    print("rows of the last conv:", voc.rows)


if __name__ == "__main__":
    main()
