"""Debug build (ITTS_PL_TRACE=1 ITTS_PL_DBG=1, via ITTS_HIP_LIB): the per-call cue loop with the persistent
layers; after every generate, what workgroups 0 / 1 / 8 read in layer 0 of the first decode step
(key index, pad, first x^ / x / c_attn-weight / K / V words, q/k/v granules, attention output)."""
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
    gpt.pl = True
    tts.LOOKAHEAD = 0
    orig = gpt.generate
    off = int(gpt.lib.itts_gpt_pl_scratch_bytes()) - 256 - 256 * 32 * 8
    names = ["kidx", "pad0", "xh", "x", "w_qkv", "K", "V", "q", "k", "v", "o"]

    def gen(*a, **k):
        out = orig(*a, **k)
        tr = gpt._pl_scratch.view(torch.uint8)[off:off + 256 * 32 * 8].view(torch.int64).view(256, 32)[:, 20:31].cpu()
        print(f"  codes[:6] = {out[0, :6].tolist()}", flush=True)
        for wg in (0, 1, 8):
            print(f"  wg {wg}: " + " ".join(f"{n}={int(v) & 0xFFFFFFFF:08x}" for n, v in zip(names, tr[wg].tolist())),
                  flush=True)
        return out
    gpt.generate = gen
    for i, t in enumerate(CUES):
        print(f"call {i}: {t!r}", flush=True)
        tts.infer(prompt, t, None, **GREEDY)


if __name__ == "__main__":
    main()
