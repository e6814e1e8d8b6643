"""Free-running greedy decode with EOS allowed (rows finishing at different steps), persistent layers vs
the launch chain, batch vs one row at a time: the long-form test's shape (8 cues, 40 codes, duplicated
rows) on the full IndexTTS-1.5 GPT."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "index-tts-dubbing_amd"))
os.environ["ITTS_PL"] = "1"
from indextts.gpt.engine import HipGPT  # noqa: E402
from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import gpt_state_dict  # noqa: E402


def stops(codes, stop):
    out = []
    for r in codes.tolist():
        out.append(r.index(stop) if stop in r else len(r))
    return out


def main():
    cfg = load_config(default_config_path())
    eng = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.08), cfg.gpt, "cuda", dtype="bf16")
    g = torch.Generator().manual_seed(11)
    B, L = 8, 20
    lens = [6, 14, 9, 6, 20, 4, 12, 16]
    base = torch.randn(1, 32, 1024, generator=g)
    conds = base.repeat(B, 1, 1).cuda()
    rows = [torch.randint(2, 12000, (n,), generator=g) for n in lens]
    rows[3] = rows[0].clone()
    text = torch.stack([torch.nn.functional.pad(r, (0, L - r.numel()), value=1) for r in rows]).cuda()
    res = {}
    for pl in (True, False):
        eng.pl = pl
        for k in list(eng._lanes):
            del eng._lanes[k]
        for mult in (1, 4):
            eng.GRAPH_STEPS = mult
            c = eng.generate(conds, text, 40, repetition_penalty=10.0).cpu()
            res[(pl, "batch", mult)] = c
            print(f"PL={pl} graph_steps={mult} batch stops: {stops(c, eng.stop_mel)} err={eng.pl_error()}", flush=True)
        singles = []
        for i in range(B):
            c = eng.generate(conds[i:i + 1], text[i:i + 1, :lens[i]], 40, repetition_penalty=10.0).cpu()
            singles.append(c)
        print(f"PL={pl} single stops: {[stops(c, eng.stop_mel)[0] for c in singles]}", flush=True)
        res[(pl, "single")] = singles
    for i in range(B):
        a, b = res[(True, "single")][i][0], res[(False, "single")][i][0]
        n = min(a.numel(), b.numel())
        d = (a[:n] != b[:n]).nonzero()
        print(f"row {i}: PL vs chain single first diff {int(d[0]) if d.numel() else None}")
    for i in range(B):
        a = res[(True, "batch", 4)][i]
        b = res[(False, "batch", 4)][i]
        n = min(a.numel(), b.numel())
        d = (a[:n] != b[:n]).nonzero()
        print(f"row {i}: PL vs chain batch first diff {int(d[0]) if d.numel() else None}")


if __name__ == "__main__":
    main()
