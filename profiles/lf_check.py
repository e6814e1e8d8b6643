"""Pass/fail probe for the persistent-layer lane-reuse bug (tests/test_gpu_longform.py's per-call cue loop):
the chain per call, then two per-call passes with the persistent layers; prints the cues whose PCM differ
from the chain in each pass.  Run against a library variant with ITTS_HIP_LIB."""
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
    d = tempfile.mkdtemp()
    cfg_path = write_checkpoint_dir(d, load_config(default_config_path()),
                                    os.path.join(HERE, "..", "tests", "golden", "tiny_bpe.model"), seed=0,
                                    mel_head_std=0.08)
    _write_prompt(os.path.join(d, "prompt.wav"))
    tts = IndexTTS(cfg_path=cfg_path, model_dir=d, is_fp16=True, device="cuda:0")
    prompt = os.path.join(d, "prompt.wav")
    gpt = tts.gpt
    tts.LOOKAHEAD = 0

    def run(pl):
        gpt.pl = pl
        for k in list(gpt._lanes):
            del gpt._lanes[k]
        return [tts.infer(prompt, t, None, **GREEDY)[1] for t in CUES]
    ref = run(False)
    res = []
    for _ in range(3):
        got = run(True)
        res.append([i for i, (a, b) in enumerate(zip(got, ref)) if not (a.shape == b.shape and np.array_equal(a, b))])
    print(f"LIB {os.path.basename(os.environ.get('ITTS_HIP_LIB', 'default'))}: differing cues per PL pass {res} "
          f"err={gpt.pl_error()}", flush=True)


if __name__ == "__main__":
    main()
