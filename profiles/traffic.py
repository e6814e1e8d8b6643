"""Per-launch HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs).

FETCH_SIZE and WRITE_SIZE (KiB per dispatch) do not fit in one TCC pass on gfx950.  Per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section), gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.

usage:
  python profiles/traffic.py vocoder <fetch_dir> <write_dir>
      igemm_kernel dispatches of the second of two vocoder forwards (profiles/pmc_vocoder.py)
  python profiles/traffic.py calibrate <fetch_dir>
      measured FETCH_SIZE of the known-byte c_fc GEMM dispatches (profiles/pmc_calibrate.py) / their
      weight bytes: ~0.5 confirms the x2 correction for this access pattern
  python profiles/traffic.py decode <fetch_dir> <write_dir>
      the GPT decode-step kernels (profiles/pmc_decode.py), summed per step; one step = one
      advance_kernel dispatch; dispatches before the first attn_decode_kernel (prefill) skipped
-> JSON on stdout
"""
import csv
import glob
import json
import os
import re
import sys

DECODE_KERNELS = ("attn_decode_kernel", "decode_gemm_kernel", "decode_gemm16_kernel", "decode_gemm16x_kernel",
                  "residual_reduce_ln", "sample_embed_kernel", "sample_topk_embed_kernel", "advance_kernel",
                  "gpt_layer_pl_kernel", "pl_zero_kernel",  # persistent layers (r04) + the per-step counter reset
                  "beam_cand_kernel", "beam_select_kernel")


def load(d, counter):
    """-> {dispatch_id: (kernel_name, value)}"""
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        name, v = vals.get(k, (r["Kernel_Name"], 0.0))
        vals[k] = (name, v + float(r["Counter_Value"]))
    return vals


def short(name):
    for k in sorted(DECODE_KERNELS, key=len, reverse=True) + ["igemm256_kernel", "igemm_kernel", "amp_conv_kernel",
                                                              "aa_snakebeta_kernel",
                                                              "aa_snake_mfma_kernel", "act_post_conv_kernel"]:
        if k in name:
            return k
    return name.split("(")[0][-40:]


def vocoder(fetch, write):
    out = {"kernel": "igemm_kernel (BigVGAN convs, second of two C3 vocoder forwards)"}
    groups = {"igemm_kernel": lambda n: "igemm_kernel" in n or "igemm256_kernel" in n,  # both tile families
              "amp_conv_kernel": lambda n: "amp_conv_kernel" in n,  # conv-only and act-fused forms
              # the activation: MFMA kernel on the vocoder's bf16 channel-last layout (VALU kernel otherwise)
              "aa_snakebeta_kernel": lambda n: "aa_snakebeta_kernel" in n or "aa_snake_mfma_kernel" in n,
              # round 6: activation_post + conv_post + tanh + int16 in one launch
              "act_post_conv_kernel": lambda n: "act_post_conv_kernel" in n}
    for name, match in groups.items():
        ids = sorted(k for k, (n, _) in fetch.items() if match(n) and k in write)
        ids = ids[len(ids) // 2:]
        if not ids:
            continue
        fb = sum(2 * 1024 * fetch[i][1] for i in ids) / len(ids)  # KiB -> bytes, x2 gfx950 correction
        wb = sum(1024 * write[i][1] for i in ids) / len(ids)
        out[name] = {"dispatches": len(ids), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                     "bytes_per_launch": fb + wb}
    out["igemm_bytes_per_launch"] = out.get("igemm_kernel", {}).get("bytes_per_launch")
    out["amp_conv_bytes_per_launch"] = out.get("amp_conv_kernel", {}).get("bytes_per_launch")
    out["aa_snakebeta_bytes_per_launch"] = out.get("aa_snakebeta_kernel", {}).get("bytes_per_launch")
    out["act_post_conv_bytes_per_launch"] = out.get("act_post_conv_kernel", {}).get("bytes_per_launch")
    out["correction"] = "FETCH_SIZE x2 (gfx950 coalesced-read undercount); KiB -> bytes"
    return out


def decode(fetch, write):
    ids = sorted(k for k, (n, _) in fetch.items() if k in write)
    first = min(k for k in ids if "attn_decode_kernel" in fetch[k][0] or "gpt_layer_pl_kernel" in fetch[k][0])
    ids = [k for k in ids if k >= first and any(s in fetch[k][0] for s in DECODE_KERNELS)]
    steps = sum(1 for k in ids if "advance_kernel" in fetch[k][0])
    per = {}
    for k in ids:
        n = short(fetch[k][0])
        f, w, c = per.get(n, (0.0, 0.0, 0))
        per[n] = (f + 2 * 1024 * fetch[k][1], w + 1024 * write[k][1], c + 1)
    tot_f = sum(v[0] for v in per.values()) / steps
    tot_w = sum(v[1] for v in per.values()) / steps
    return {"kernel": "GPT decode step (all decode-step dispatches, graph disabled)", "steps": steps,
            "fetch_bytes_per_step": tot_f, "write_bytes_per_step": tot_w, "bytes_per_step": tot_f + tot_w,
            "per_kernel_per_step": {n: {"launches": c // steps, "fetch_bytes": f / steps, "write_bytes": w / steps}
                                    for n, (f, w, c) in per.items()},
            "correction": "FETCH_SIZE x2 (gfx950 coalesced-read undercount); KiB -> bytes"}


def calibrate(fetch):
    weight_bytes = 4096 * 1024 * 2
    ids = sorted(k for k, (n, _) in fetch.items() if "decode_gemm16x_kernel" in n)
    raw = [1024 * fetch[k][1] for k in ids[2:]]  # skip the first (cold code / TLB) dispatches
    mean = sum(raw) / len(raw)
    return {"kernel": "decode_gemm16x_kernel, N=4096 K=1024 M=32 (c_fc shape), distinct weight copies",
            "dispatches": len(raw), "weight_bytes": weight_bytes, "fetch_size_bytes_per_dispatch": mean,
            "ratio_fetch_size_to_weight_bytes": mean / weight_bytes,
            "note": "ratio ~0.5 = FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads (x2 correction)"}


def main():
    if sys.argv[1] == "calibrate":
        print(json.dumps(calibrate(load(sys.argv[2], "FETCH_SIZE")), indent=1))
        return
    mode, fdir, wdir = sys.argv[1:4]
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    print(json.dumps(vocoder(fetch, write) if mode == "vocoder" else decode(fetch, write), indent=1))


if __name__ == "__main__":
    main()
