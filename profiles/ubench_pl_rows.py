"""Greedy decode time per step at several row counts, persistent layers vs the launch chain (one engine; the
chain forced with HipGPT.launch_chain()): 400 steps after a 48-id text and 32 conditioning frames (the C3 /
C5 shape), seeded synthetic weights, HIP events around generate(), median of 3 runs.
Prints `rows <R> pl <us> chain <us>` per row count (argv: row counts, default 32 64 96 128)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "index-tts-dubbing_amd"))
from indextts.gpt.engine import HipGPT  # noqa: E402
from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import gpt_state_dict  # noqa: E402

STEPS = int(os.environ.get("STEPS", "400"))


def timed(eng, conds, text, chain):
    ts = []
    for i in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        if chain:
            with eng.launch_chain():
                eng.generate(conds, text, STEPS, min_new_tokens=STEPS)
        else:
            eng.generate(conds, text, STEPS, min_new_tokens=STEPS)
        b.record()
        torch.cuda.synchronize()
        if i > 0:
            ts.append(a.elapsed_time(b) * 1e3 / STEPS)
    return sorted(ts)[1]


def main():
    cfg = load_config(default_config_path())
    eng = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.08), cfg.gpt, "cuda", dtype="bf16", max_kv=512)
    eng.PL_MAX_ROWS = 128
    for R in [int(v) for v in (sys.argv[1:] or ["32", "64", "96", "128"])]:
        g = torch.Generator().manual_seed(R)
        text = torch.randint(2, 12000, (R, 48), generator=g).cuda()
        conds = torch.randn(R, 32, 1024, generator=g).cuda()
        assert eng.pl_takes(R), R
        pl = timed(eng, conds, text, False)
        ch = timed(eng, conds, text, True)
        print(f"rows {R} pl {pl:.1f} chain {ch:.1f} us per step (generate incl. prefill)", flush=True)


if __name__ == "__main__":
    main()
