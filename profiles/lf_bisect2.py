"""Hypotheses for the persistent-layer mismatch on a reused decode lane (profiles/lf_bisect.py): record
the cue loop's 8 generate calls (chain), then per variant run them twice with the persistent layers on
fresh lanes and compare the second pass with the chain: zero the PL scratch before every call, zero the
lane KV caches, or zero the x^ rows past the batch."""
import os
import sys
import tempfile

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("ITTS_PL", "1")  # build the persistent-layer operands (opt-in path)
sys.path.insert(0, os.path.join(HERE, "..", "index-tts-dubbing_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from test_gpu_longform import CUES, GREEDY, _write_prompt  # noqa: E402


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
    tts.LOOKAHEAD = 0
    rec = []
    orig = gpt.generate

    def hook(conds, ids, n, **kw):
        out = orig(conds, ids, n, **kw)
        rec.append((conds.clone(), ids.clone(), n, dict(kw), out.cpu().clone()))
        return out
    gpt.pl = False
    gpt.generate = hook
    for t in CUES:
        tts.infer(prompt, t, None, **GREEDY)
    gpt.generate = orig

    def lanes_state():
        return [v["st"] for k, v in gpt._lanes.items() if isinstance(k, tuple) and len(k) == 2 and isinstance(v, dict)]

    def variant(label, before=None):
        gpt.pl = True
        for k in list(gpt._lanes):
            del gpt._lanes[k]
        bad = None
        for rep in range(2):
            bad = []
            for i, (conds, ids, n, kw, want) in enumerate(rec):
                if before is not None:
                    before()
                got = orig(conds, ids, n, **kw).cpu()
                m = min(got.shape[1], want.shape[1])
                dd = (got[:, :m] != want[:, :m]).nonzero()
                if dd.numel() or got.shape != want.shape:
                    bad.append((i, int(dd[0][1]) if dd.numel() else "len"))
        print(f"{label:30s} second pass differing calls (call, first step): {bad}", flush=True)

    def zero_scratch():
        gpt._pl_scratch.zero_()

    def zero_kv():
        for st in lanes_state():
            st["kc"].zero_()
            st["vc"].zero_()

    def zero_h_pad():
        for st in lanes_state():
            st["h"][st["B"]:].zero_()

    variant("baseline")
    variant("zero PL scratch per call", zero_scratch)
    variant("zero lane KV per call", zero_kv)
    variant("zero x^ rows >= B per call", zero_h_pad)


if __name__ == "__main__":
    main()
