"""Phase timeline of one persistent decode layer (gpt_layer.hip built with -DITTS_PL_TRACE=1, loaded via
ITTS_HIP_LIB): decode a C3-shaped batch greedily, then read the 100-MHz stamps wave 0 of every
workgroup wrote at the phase boundaries of layer ITTS_PL_TRACE_LAYER of the last step.  Prints, per
mark, the spread over the 256 workgroups relative to the earliest kernel start (µs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "index-tts-dubbing_amd"))
os.environ["ITTS_PL"] = "1"
from indextts.gpt.engine import HipGPT  # noqa: E402
from indextts.utils.config import default_config_path, load_config  # noqa: E402
from indextts.utils.synthetic import gpt_state_dict  # noqa: E402

NAMES = ["start", "A0 issued", "A c_attn", "E1 q/k/v in", "B attention", "E2 o ready", "C c_proj",
         "E3 part ready", "D x1", "E4 x1 ready", "E c_fc", "E5 f ready", "F mlp.c_proj", "E6 part ready",
         "G end", "E2 drained", "E3 drained", "E4 drained", "E5 drained", "E6 drained", "B keys done",
         "B round 0 done"]


def run(eng, B, L_text=48, steps=int(os.environ.get("STEPS", "40"))):
    g = torch.Generator().manual_seed(3)
    text = torch.randint(2, 12000, (B, L_text), generator=g).cuda()
    conds = torch.randn(B, 32, 1024, generator=g).cuda()
    for k in list(eng._lanes):
        del eng._lanes[k]
    nb = int(os.environ.get("BEAMS", "1"))  # BEAMS=3: B / 3 utterances, beam search (B rows)
    if nb > 1:
        eng.generate(conds[: B // nb], text[: B // nb], steps, min_new_tokens=steps, num_beams=nb)
    else:
        eng.generate(conds, text, steps, min_new_tokens=steps)
    torch.cuda.synchronize()
    OFF_TRACE = int(eng.lib.itts_gpt_pl_scratch_bytes()) - 256 - 256 * 32 * 8  # trace, then the epoch / error block
    tr = eng._pl_scratch.view(torch.uint8)[OFF_TRACE:OFF_TRACE + 256 * 32 * 8].view(torch.int64).view(256, 32)
    tr = tr[:, :22].cpu().double()
    t0 = tr[:, 0].min()
    rel = (tr - t0) / 100.0  # 100 MHz -> µs
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(rel.clone(), f"gpurun_out/pl_trace_raw_B{B}_{steps}.pt")
    print(f"B={B}, {steps} steps (keys at the traced step: {32 + L_text + 2 + steps}): layer span {float(rel[:, 14].max()):.2f} us (first start -> last end)")
    prev = None
    order = [0, 1, 2, 3, 21, 20, 4, 15, 5, 6, 16, 7, 8, 17, 9, 10, 18, 11, 12, 19, 13, 14]
    for i in order:
        n = NAMES[i]
        col = rel[:, i]
        ok = col.abs() < 1e6  # D's marks (7, 8, 17) are stamped by the tile owners only (round 6)
        cv = col[ok]
        if cv.numel() == 0:  # a mark this build does not stamp
            prev = None
            continue
        line = f"  {i:2d} {n:14s} min {float(cv.min()):7.2f} med {float(cv.median()):7.2f} max {float(cv.max()):7.2f}"
        if int(ok.sum()) < 256:
            line += f" ({int(ok.sum())} WGs)"
        if prev is not None:
            d = (col - prev)[ok & (prev.abs() < 1e6)]
            if d.numel():
                line += f"   | per-WG dt med {float(d.median()):6.2f} max {float(d.max()):6.2f}"
        print(line, flush=True)
        prev = col
    # hand-off protocol latency per edge: the last producer's add (after its drain) -> each consumer's poll
    # match.  Cluster edges (E2, E4, E5): producers and consumers = the 32 workgroups b % 8 == c; tile edges
    # (E3, E6): the 8 workgroups of tile j = b / 8
    b = torch.arange(256)
    for name, m_add, m_rdy, key in (("E2", 15, 5, b % 8), ("E3", 16, 7, b // 8), ("E4", 17, 9, b % 8),
                                    ("E5", 18, 11, b % 8), ("E6", 19, 13, b // 8)):
        lat = []
        for k in key.unique():
            sel = key == k
            add, rdy = rel[sel, m_add], rel[sel, m_rdy]
            add, rdy = add[add.abs() < 1e6], rdy[rdy.abs() < 1e6]
            if add.numel() and rdy.numel():
                lat.append(rdy - add.max())
        if not lat:
            continue
        lat = torch.cat(lat)
        print(f"  {name}: last add -> ready  min {float(lat.min()):5.2f} med {float(lat.median()):5.2f} "
              f"max {float(lat.max()):5.2f} us", flush=True)


if __name__ == "__main__":
    cfg = load_config(default_config_path())
    eng = HipGPT(gpt_state_dict(cfg.gpt, 0, 0.08), cfg.gpt, "cuda", dtype="bf16", max_kv=512)
    for B in [int(v) for v in (sys.argv[1:] or ["32", "1"])]:
        run(eng, B)
