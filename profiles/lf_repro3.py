"""Record every HipGPT.generate call of the per-call cue loop (persistent layers on, fresh engine), then
replay the recorded inputs: chain, PL on fresh lanes, PL on the warm lanes; print per call the first
step whose id differs from the recorded PL run."""
import os
import sys
import tempfile

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("ITTS_PL", "1")  # build the persistent-layer operands (opt-in path)
sys.path.insert(0, os.path.join(HERE, "..", "index-tts-dubbing_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from test_gpu_longform import CUES, GREEDY, _write_prompt  # noqa: E402


def first_diff(a, b):
    n = min(a.shape[1], b.shape[1])
    d = (a[:, :n] != b[:, :n]).nonzero()
    return (int(d[0][1]) if d.numel() else None), tuple(a.shape), tuple(b.shape)


def main():
    from indextts.infer import IndexTTS
    from indextts.utils.config import default_config_path, load_config
    from indextts.utils.synthetic import write_checkpoint_dir
    d = tempfile.mkdtemp()
    cfg_path = write_checkpoint_dir(d, load_config(default_config_path()),
                                    os.path.join(HERE, "..", "tests", "golden", "tiny_bpe.model"), seed=0,
                                    mel_head_std=0.08)
    _write_prompt(os.path.join(d, "prompt.wav"))
    tts = IndexTTS(cfg_path=cfg_path, model_dir=d, is_fp16=True, device="cuda:0")
    prompt = os.path.join(d, "prompt.wav")
    gpt = tts.gpt
    rec = []
    orig = gpt.generate

    def hook(conds, ids, n, **kw):
        out = orig(conds, ids, n, **kw)
        rec.append((conds.clone(), ids.clone(), n, dict(kw), out.cpu().clone(), gpt.pl_error()))
        return out
    gpt.generate = hook
    tts.LOOKAHEAD = 0
    for t in CUES:
        tts.infer(prompt, t, None, **GREEDY)
    gpt.generate = orig
    print("recorded calls:", [(tuple(r[1].shape), r[2], tuple(r[4].shape), r[5]) for r in rec], flush=True)
    for mode in ("chain", "pl_fresh", "pl_warm"):
        gpt.pl = mode != "chain"
        if mode != "pl_warm":
            for k in list(gpt._lanes):
                del gpt._lanes[k]
        res = []
        for conds, ids, n, kw, out, _ in rec:
            res.append(first_diff(orig(conds, ids, n, **kw).cpu(), out))
        print(mode, res, flush=True)


if __name__ == "__main__":
    main()
