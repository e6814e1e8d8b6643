"""tests/test_gpu_longform.py's flow with per-cue diagnostics: per-call and lookahead synthesis of the 8
cues with the persistent decode layers on and off (same IndexTTS object), printing each cue's raw code
count and whether its PCM equals the per-call chain result."""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("ITTS_PL", "1")  # build the persistent-layer operands (opt-in path)
sys.path.insert(0, os.path.join(HERE, "..", "index-tts-dubbing_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from test_gpu_longform import CUES, GREEDY, _write_prompt  # noqa: E402
from test_gpu_lookahead import _Entry  # noqa: E402


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
    res = {}
    for pl in ((True, False) if os.environ.get("PL_FIRST") else (False, True)):
        tts.gpt.pl = pl
        tts.LOOKAHEAD = 0
        res[(pl, "call")] = [tts.infer(prompt, t, None, **GREEDY)[1] for t in CUES]
        print(f"PL={pl} per-call samples: {[w.size for w in res[(pl, 'call')]]}", flush=True)
        tts.LOOKAHEAD = 128
        entries = [_Entry(i + 1, t) for i, t in enumerate(CUES)]
        out = []
        for i, entry in enumerate(entries):
            out.append(tts.infer(prompt, entry.text, None, **GREEDY)[1])
        res[(pl, "look")] = out
        print(f"PL={pl} lookahead samples: {[w.size for w in out]}", flush=True)
    ref = res[(False, "call")]
    for key, v in res.items():
        eq = [bool(a.shape == b.shape and np.array_equal(a, b)) for a, b in zip(v, ref)]
        print(f"{key}: equal to chain per-call: {eq}", flush=True)


if __name__ == "__main__":
    main()
