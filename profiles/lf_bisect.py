"""Bisect the persistent-layer mismatch of the per-call cue loop (tests/test_gpu_longform.py): the 8 cues
per call with the chain (reference), then with the persistent layers under variants of the decode
driver, each on fresh decode lanes; prints which cues' PCM differ from the chain."""
import os
import sys
import tempfile

import numpy as np
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
    orig_gen = gpt.generate

    def run(label, pl, graph_steps=4, sync=False, max_shapes=4, use_graph=True, between=None):
        gpt.pl = pl
        gpt.GRAPH_STEPS = graph_steps
        gpt.MAX_CACHED_SHAPES = max_shapes
        for k in list(gpt._lanes):
            del gpt._lanes[k]

        def gen(*a, **k):
            if sync:
                torch.cuda.synchronize()
            k.setdefault("use_graph", use_graph)
            return orig_gen(*a, **k)
        gpt.generate = gen
        out = []
        for t in CUES:
            out.append(tts.infer(prompt, t, None, **GREEDY)[1])
            if between is not None:
                between()
        gpt.generate = orig_gen
        return out

    def lanes_state():
        return [v["st"] for k, v in gpt._lanes.items() if isinstance(k, tuple) and len(k) == 2 and isinstance(v, dict)]

    def zero_scratch():
        gpt._pl_scratch.zero_()

    nb = int(gpt.lib.itts_gpt_pl_scratch_bytes())
    p2 = nb - 256 - 256 * 32 * 8 - 8 * 128 * 1024 * 4
    fc = p2 - 8 * 128 * 512 * 2
    xc = fc - 8 * 128 * 1024 * 2
    p1 = xc - 8 * 128 * 1024 * 4
    ob = p1 - 8 * 128 * 128 * 2
    gq = ob - 128 * 16 * 192 * 8
    sc = gpt._pl_scratch.view(torch.uint8)

    def zero_range(a, b):
        return lambda: sc[a:b].zero_()

    def zero_kv():
        for st in lanes_state():
            st["kc"].zero_()
            st["vc"].zero_()

    def zero_bufs():
        for st in lanes_state():
            for k in ("x", "h", "logits"):
                st[k].zero_()

    def pre(fn):  # run fn before every generate
        def gen(*a, **k):
            fn()
            return orig_gen(*a, **k)
        return gen

    def run_with(label, gen):
        gpt.pl = True
        for k in list(gpt._lanes):
            del gpt._lanes[k]
        gpt.generate = gen
        out = [tts.infer(prompt, t, None, **GREEDY)[1] for t in CUES]
        gpt.generate = orig_gen
        return out

    ref = run("chain", False)
    variants = [("pl", {}, None), ("pl again", {}, None), ("pl zero counters", {}, zero_range(0, gq)),
                ("pl zero granules", {}, zero_range(gq, ob)), ("pl zero ob..p2", {}, zero_range(ob, p2 + 8 * 128 * 1024 * 4)),
                ("pl zero trace/err", {}, zero_range(p2 + 8 * 128 * 1024 * 4, nb)), ("pl zero scratch", {}, zero_scratch)]
    for label, kw, fn in variants:
        if fn is not None:
            orig_gen_saved = orig_gen
            gpt_gen = pre(fn)
            got = run_with(label, gpt_gen)
        else:
            got = run(label, True, **kw)
        bad = [i for i, (a, b) in enumerate(zip(got, ref)) if not (a.shape == b.shape and np.array_equal(a, b))]
        print(f"{label:28s} differing cues: {bad}  err={gpt.pl_error()}", flush=True)


if __name__ == "__main__":
    main()
