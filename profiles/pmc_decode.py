"""Workload for the rocprofv3 PMC passes over the GPT decode step (HBM traffic per step).

Runs bench.py's C3 GPT decode kernels (B=32 utterances, random-init IndexTTS-1.5 weights, bf16) for
``STEPS`` forced steps with the hipGraph disabled, so every decode-step kernel is an ordinary dispatch
that the counter passes attribute one by one (the kernels are the ones the graph replays).  The
counter passes crash the profiler (host SIGSEGV) at C3's 400 steps x 143 dispatches, so the run is
96 steps long and the text is lengthened (L=200) so that the mean number of keys attended per row,
s + 2 + (STEPS - 2)/2 = 283, equals C3's (L=48 over 400 steps): bytes per step then compare
directly with bench.py's algorithmic bytes per step.  ``profiles/traffic.py decode`` sums the per-dispatch bytes of the decode-step kernels
and divides by the number of steps.

    cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_f -o run -- python profiles/pmc_decode.py
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc_w -o run -- python profiles/pmc_decode.py
    python profiles/traffic.py decode /tmp/pmc_f /tmp/pmc_w
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "index-tts-dubbing_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from indextts.gpt.engine import HipGPT  # noqa: E402
from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import gpt_state_dict  # noqa: E402

B, L, STEPS = 32, 200, 96
BEAM3 = len(sys.argv) > 1 and sys.argv[1] == "beam3"  # the reference's default decoding: 3 beams x 32


def _heartbeat():
    """a line every 30 s: counter passes over the 96-row beam step run for minutes without output"""
    import threading
    import time

    def beat():
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"[pmc_decode] running {time.time() - t0:.0f} s", flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    _heartbeat()
    cfg = load_config(default_config_path())
    eng = HipGPT(gpt_state_dict(cfg.gpt, seed=0, mel_head_std=0.08), cfg.gpt, "cuda", "bf16",
                 max_kv=32 + L + 2 + 1 + STEPS + 8)
    g = np.random.default_rng(2)
    conds = torch.from_numpy(g.normal(0, 1, (B, 32, eng.D)).astype(np.float32)).cuda()
    text = torch.from_numpy(g.integers(2, 12000, (B, L))).cuda()
    if BEAM3:
        codes = eng.generate(conds, text, STEPS, min_new_tokens=STEPS, use_graph=False, check_every=10 ** 9,
                             num_beams=3, do_sample=True, top_k=30, top_p=0.8, seed=1234)
    else:
        codes = eng.generate(conds, text, STEPS, min_new_tokens=STEPS, use_graph=False, check_every=10 ** 9)
    torch.cuda.synchronize()
    s = 32 + L + 2
    print(f"decode steps: {STEPS - 1} (after prefill), beam3 {BEAM3}, persistent layers {eng.pl}, codes {tuple(codes.shape)}, "
          f"mean keys per row {s + 2 + (STEPS - 2) / 2:.1f} (= bench.py C3)")


if __name__ == "__main__":
    main()
