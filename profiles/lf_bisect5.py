"""Size of the persistent-layer deviation on a reused decode lane: the cue loop per call with raw-logit
tracing, chain vs persistent layers (second PL pass, where cue 3 deviates), per call the first step whose
logits differ and by how much."""
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
    orig = gpt.generate
    traces = {}

    def run(label, pl):
        gpt.pl = pl
        for k in list(gpt._lanes):
            del gpt._lanes[k]
        calls = []

        def gen(*a, **k):
            gpt.logits_trace = []
            out = orig(*a, **k)
            calls.append([t.cpu() for t in gpt.logits_trace])
            gpt.logits_trace = None
            return out
        gpt.generate = gen
        for t in CUES:
            tts.infer(prompt, t, None, **GREEDY)
        gpt.generate = orig
        traces[label] = calls

    run("chain", False)
    run("pl1", True)
    run("pl2", True)
    for label in ("pl1", "pl2"):
        for i, (a, b) in enumerate(zip(traces[label], traces["chain"])):
            first = None
            for s, (x, y) in enumerate(zip(a, b)):
                if not torch.equal(x, y):
                    dd = (x - y).abs()
                    first = (s, int((x != y).sum()), float(dd.max()), float(y.abs().max()))
                    break
            print(f"{label} call {i}: steps {len(a)}/{len(b)} first differing step (step, n, max|d|, max|ref|): {first}",
                  flush=True)


if __name__ == "__main__":
    main()
