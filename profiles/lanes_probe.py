"""Concurrent decode chains on CU-partitioned streams: C3-shaped greedy decode (400 steps) of
  A: one 32-row batch, one lane (the product path),
  B: two 32-row batches as two lanes on unmasked streams,
  C: the same two lanes on disjoint CU halves (hipExtStreamCreateWithCUMask, 16 CUs per XCD each),
  D: one 32-row batch as two 16-row lanes on disjoint halves.
Decode on 128 CUs alone runs as fast as on 256 (profiles/cumask_probe_r02.txt): the chain is
latency-bound, so two chains might share the chip.  Prints ms and ms per 32 rows."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd")]
import torch

from bench import make_inputs
from indextts.pipeline import BatchedTTS
from indextts.utils.config import default_config_path, load_config
from indextts.utils.synthetic import bigvgan_state_dict, gpt_state_dict

hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(0).multi_processor_count


def masked_stream(bits):
    words = (ctypes.c_uint32 * ((NCU + 31) // 32))()
    for i in bits:
        words[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), len(words), words) == 0
    return torch.cuda.ExternalStream(h.value)


def main():
    dev = torch.device("cuda:0")
    cfg = load_config(default_config_path())
    N, L = 400, 48
    tts = BatchedTTS(gpt_state_dict(cfg.gpt, seed=0, mel_head_std=0.08), bigvgan_state_dict(cfg.bigvgan, seed=0),
                     cfg, dev, "bf16", max_kv=32 + L + 2 + 1 + N + 8)
    mels, texts = make_inputs(cfg, list(range(128)), L, 511)
    mels = [m.to(dev) for m in mels]
    conds, _ = tts.prompt_features(mels, None)
    ids = torch.full((128, L), tts.stop_text, dtype=torch.long)
    for b, t in enumerate(texts):
        ids[b, : t.numel()] = t.reshape(-1).long()
    ids = ids.to(dev)
    gpt = tts.gpt
    lo = [i for i in range(NCU) if i % 32 < 16]
    hi = [i for i in range(NCU) if i % 32 >= 16]
    plain = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    masked = [masked_stream(lo), masked_stream(hi)]

    def run(rows, lanes, streams, note):
        gpt._lanes = {}  # fresh lane states / graphs bound to these streams
        for i, s in enumerate(streams):
            gpt._lanes[("stream", i)] = s
        ref = None
        for rep in range(2):  # the first call captures the graphs
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            codes = gpt.generate(conds[:rows], ids[:rows], N, repetition_penalty=10.0, min_new_tokens=N, lanes=lanes)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            ref = codes if ref is None else ref
        print(f"{note:44s} {dt:8.1f} ms  {dt * 32 / rows:8.1f} ms per 32 rows", flush=True)
        return codes

    a = run(32, 1, plain[:1], "A 32 rows, 1 lane, all CUs")
    b = run(64, 2, plain, "B 64 rows, 2 lanes x 32, all CUs")
    c = run(64, 2, masked, "C 64 rows, 2 lanes x 32, CU halves")
    d = run(32, 2, masked, "D 32 rows, 2 lanes x 16, CU halves")
    quarters = [masked_stream([i for i in range(NCU) if 8 * q <= i % 32 < 8 * q + 8]) for q in range(4)]
    thirds = [masked_stream([i for i in range(NCU) if lo_ <= i % 32 < hi_]) for lo_, hi_ in ((0, 11), (11, 22), (22, 32))]
    run(64, 1, plain[:1], "H 64 rows, 1 lane, all CUs")
    run(128, 1, plain[:1], "I 128 rows, 1 lane, all CUs")
    run(96, 3, thirds, "E 96 rows, 3 lanes x 32, CU thirds")
    run(128, 4, quarters, "F 128 rows, 4 lanes x 32, CU quarters")
    run(128, 2, masked, "G 128 rows, 2 lanes x 64, CU halves")
    run(64, 4, quarters, "J 64 rows, 4 lanes x 16, CU quarters")
    print("ids equal A vs C rows 0-31:", bool(torch.equal(a, c[:32, : a.shape[1]])), flush=True)


if __name__ == "__main__":
    main()
