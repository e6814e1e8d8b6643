"""CU-mask probe: how the C3 decode (400 hipGraph steps) and the back half (latent pass + vocoder)
run on complementary CU subsets, alone and concurrently -- the question being whether the
latency-bound decode chain can share the chip with the MFMA/VALU-heavy back half.

Streams come from hipExtStreamCreateWithCUMask (bit i of the mask = logical CU i) wrapped as
torch ExternalStreams.  Prints ms per phase for each mask configuration."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch

from bench import make_inputs
from indextts.pipeline import BatchedTTS, remove_long_silence
from indextts.utils.config import default_config_path, load_config
from indextts.utils.synthetic import bigvgan_state_dict, gpt_state_dict

hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(0).multi_processor_count


def masked_stream(bits):
    words = (ctypes.c_uint32 * ((NCU + 31) // 32))()
    for i in bits:
        words[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), len(words), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value)


def main():
    dev = torch.device("cuda:0")
    cfg = load_config(default_config_path())
    B, N, L = 32, 400, 48
    tts = BatchedTTS(gpt_state_dict(cfg.gpt, seed=0, mel_head_std=0.08), bigvgan_state_dict(cfg.bigvgan, seed=0),
                     cfg, dev, "bf16", max_kv=32 + L + 2 + 1 + N + 8)
    mels, texts = make_inputs(cfg, list(range(B)), L, 511)
    mels = [m.to(dev) for m in mels]
    texts = [t.to(dev) for t in texts]
    # one full synthesize for warm-up and for the back half's inputs
    pcm, lens, fixed = tts.synthesize(mels, texts, max_mel_tokens=N, min_new_tokens=N)
    conds, spk = tts.prompt_features(mels, None)
    ids = torch.full((B, L), tts.stop_text, dtype=torch.long)
    for b, t in enumerate(texts):
        ids[b, : t.numel()] = t.reshape(-1).long()
    ids = ids.to(dev)
    torch.cuda.synchronize()

    def front():
        return tts.gpt.generate(conds, ids, N, repetition_penalty=10.0, min_new_tokens=N)

    def back():
        latent, ln = tts.gpt.latent(conds, [t.reshape(-1) for t in texts], fixed)
        tts.vocoder.forward(latent, ln, spk)

    # timeline of the two streams when both run: events at start / end of each (ms from the start)
    def timeline(sa, sb, note):
        torch.cuda.synchronize()
        ev = {k: torch.cuda.Event(enable_timing=True) for k in ("t0", "b0", "b1", "f0", "f1")}
        ev["t0"].record()
        with torch.cuda.stream(sb):
            ev["b0"].record(sb)
            back()
            ev["b1"].record(sb)
        with torch.cuda.stream(sa):
            ev["f0"].record(sa)
            front()
            ev["f1"].record(sa)
        torch.cuda.synchronize()
        t = {k: ev["t0"].elapsed_time(v) for k, v in ev.items() if k != "t0"}
        print(f"timeline {note}: back {t['b0']:.1f}-{t['b1']:.1f}  front {t['f0']:.1f}-{t['f1']:.1f} ms", flush=True)


    # mask bits: 32 per XCD; alternating bits select every CU here (measured, profiles/cumask_check.py),
    # so split each XCD's 32 bits into contiguous ranges
    half_a = [i for i in range(NCU) if i % 32 < 16]
    half_b = [i for i in range(NCU) if i % 32 >= 16]
    quarter = [i for i in range(NCU) if i % 32 >= 24]
    three_q = [i for i in range(NCU) if i % 32 < 24]
    configs = {"all": (None, None), "half/half": (half_a, half_b), "3q/1q": (three_q, quarter)}
    for name, (fa, fb) in configs.items():
        sa = masked_stream(fa) if fa else torch.cuda.Stream(dev)
        sb = masked_stream(fb) if fb else torch.cuda.Stream(dev)
        for label, runs in (("front alone", [(sa, front)]), ("back alone", [(sb, back)]),
                            ("both", [(sb, back), (sa, front)])):
            for rep in range(2):  # first run captures graphs on the new stream
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for s, fn in runs:
                    with torch.cuda.stream(s):
                        fn()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) * 1e3
            print(f"{name:10s} {label:12s} {dt:8.1f} ms", flush=True)
        timeline(sa, sb, name)


if __name__ == "__main__":
    main()
