"""Stress probe for the persistent-layer lane-reuse issue: the long-form per-call cue loop (8 cues,
greedy, 40 codes) once on the chain as the reference, then PASSES passes with the persistent layers
(lanes kept across passes, as a serving process would); counts cues whose PCM differ from the chain."""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("ITTS_PL", "1")
sys.path.insert(0, os.path.join(HERE, "..", "index-tts-dubbing_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from test_gpu_longform import CUES, GREEDY, _write_prompt  # noqa: E402


def main():
    from indextts.infer import IndexTTS
    from indextts.utils.config import default_config_path, load_config
    from indextts.utils.synthetic import write_checkpoint_dir
    passes = int(os.environ.get("PASSES", "8"))
    d = tempfile.mkdtemp()
    cfg_path = write_checkpoint_dir(d, load_config(default_config_path()),
                                    os.path.join(HERE, "..", "tests", "golden", "tiny_bpe.model"), seed=0,
                                    mel_head_std=0.08)
    _write_prompt(os.path.join(d, "prompt.wav"))
    tts = IndexTTS(cfg_path=cfg_path, model_dir=d, is_fp16=True, device="cuda:0")
    prompt = os.path.join(d, "prompt.wav")
    gpt = tts.gpt
    tts.LOOKAHEAD = 0
    gpt.pl = False
    ref = [tts.infer(prompt, t, None, **GREEDY)[1] for t in CUES]
    gpt.pl = True
    bad = []
    for _ in range(passes):
        got = [tts.infer(prompt, t, None, **GREEDY)[1] for t in CUES]
        bad.append([i for i, (a, b) in enumerate(zip(got, ref)) if not (a.shape == b.shape and np.array_equal(a, b))])
    n = sum(len(b) for b in bad)
    print(f"LIB {os.path.basename(os.environ.get('ITTS_HIP_LIB', 'default'))}: {n} bad cues of {passes * len(CUES)}: "
          f"{bad} err={gpt.pl_error()}", flush=True)


if __name__ == "__main__":
    main()
