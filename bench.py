#!/usr/bin/env python
"""IndexTTS-1.5 hot-path throughput on MI355X: audio-seconds per wall-second (BASELINE.json metric).

One "step" = one batch of B=32 zero-shot utterances per GPU (config C3): per-prompt conditioning +
ECAPA speaker embedding for 32 distinct prompt mels (511 frames), GPT prefill + 400 greedy decode
steps (EOS suppressed, hipGraph-replayed) at repetition_penalty 10, remove_long_silence, the
teacher-forced latent pass, BigVGAN2 -> int16 PCM; with N>1 ranks the finished waveforms are gathered
to rank 0 over RCCL (utterances shard data-parallel, weak scaling).  Inputs are resident in HBM when
the timed region starts; weights are seeded random-init IndexTTS-1.5 (no checkpoints are available).

Also reports ``roofline``: the dominant unit of work, the hipGraph-replayed GPT decode step (>60 % of
the step; HBM-bound): algorithmic bytes (every weight byte + the K/V rows attended) per replay /
the replay's duration from HIP events recorded on the decode stream around each replay, and
``traffic`` = measured HBM bytes per step from the rocprofv3 FETCH_SIZE/WRITE_SIZE passes of the
current build (profiles/run_profiles_r06.sh -> the TRAFFIC_DECODE file below); ``roofline_vocoder_conv``:
the MFMA implicit GEMM running the BigVGAN convs, and the HBM-bound vocoder kernels (activation, AMP
convs, fused conv -> activation), from HIP events around each launch; and ``cpu_baseline``: the fp32
oracle (a CPU restatement of the reference path) on a bounded sample, on this host's cores.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "index-tts-dubbing_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "audio-seconds/sec/GPU (RTF) IndexTTS-1.5 bf16 batch=32; 1→8 GPU scaling"
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
# PMC traffic summaries of the CURRENT build (profiles/run_profiles.sh; FETCH_SIZE x2 per
# MI355X_MICROARCH.md, calibrated by profiles/pmc_calibrate.py); None when not yet measured
# per decoding and decode path (persistent layers or the launch chain): None until measured for this build
# PMC files are measured on the C3 workload (profiles/pmc_decode.py, pmc_vocoder.py): other workloads report
# traffic null rather than C3's bytes
TRAFFIC_DECODE = {("c3", "greedy", True): "traffic_decode_pl_r06y.json", ("c3", "greedy", False): "traffic_decode_chain_r06y.json",
                  ("c3", "beam3", True): "traffic_decode_beam3_r06y.json",
                  ("c3", "beam3", False): "traffic_decode_beam3_r05f.json"}
TRAFFIC_VOCODER = {"c3": "traffic_vocoder_r06y.json"}


class KernelTimer:
    """HIP-event timing of every launch of one kernel family, on the stream it is launched on."""

    def __init__(self):
        self.events = []
        self.flops = 0.0
        self.bytes = 0.0
        self.launches = 0
        self.enabled = False

    def wrap(self, fn, flops, nbytes=0.0):
        if not self.enabled:
            return fn()
        s = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        r = fn()
        b.record(s)
        self.events.append((a, b))
        self.flops += flops
        self.bytes += nbytes
        self.launches += 1
        return r

    def result(self):
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in self.events)
        return ms, self.flops, self.launches


def install_conv_timer(voc, timer):
    orig = voc._conv

    def timed(c, x, y, lens, **kw):
        rows = voc.rows  # host-side count of valid rows (no device sync)
        # algorithmic bytes: valid input rows read once, output rows written once, residual rows read,
        # the packed weights read once (bf16)
        nres = sum(kw.get(k) is not None for k in ("r1", "r2"))
        nbytes = 2.0 * rows * (c.cin + c.cout * (1 + nres)) + 2.0 * c.ntaps * c.cin * c.cout
        return timer.wrap(lambda: orig(c, x, y, lens, **kw), 2.0 * rows * c.cout * c.cin * c.ntaps, nbytes)

    voc._conv = timed


def install_hbm_timers(voc, t_act, t_amp, t_tail):
    """HIP events around the standalone activation launches, the AMPBlock1 conv launches (itts_amp_conv_fwd,
    C = 24 / 48 / 96, conv-only or with the activation fused) and the generator's tail (activation_post + conv_post
    + tanh + int16, itts_act_conv_post_tanh), with their algorithmic HBM bytes: valid rows x channels, each element
    read once and written once (+ residual rows read; + the packed weights once; the tail: its input once, the f32
    waveform and the int16 PCM written once)."""
    orig_act, orig_amp, orig_tail = voc._act, voc._amp, voc._tail

    def act(a, x, y, lens):
        nbytes = 2.0 * voc.rows * x.shape[2] * 2
        return t_act.wrap(lambda: orig_act(a, x, y, lens), 0.0, nbytes)

    def amp(c, x, y, lens, a=None, r1=None, r2=None, alpha=1.0):
        nres = (r1 is not None) + (r2 is not None)
        nbytes = 2.0 * voc.rows * (c.cin + c.cout * (1 + nres)) + 2.0 * c.ntaps * c.cin * c.cout
        return t_amp.wrap(lambda: orig_amp(c, x, y, lens, a, r1, r2, alpha), 2.0 * voc.rows * c.cout * c.cin * c.ntaps,
                          nbytes)

    def tail(x, lens, wav, pcm, fused=None):
        nbytes = 2.0 * voc.rows * x.shape[2] + voc.rows * (4.0 + (2.0 if pcm is not None else 0.0))
        return t_tail.wrap(lambda: orig_tail(x, lens, wav, pcm, fused), 0.0, nbytes)

    voc._act, voc._amp, voc._tail = act, amp, tail


def _traffic(name, key):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (profiles/run_profiles_r05.sh)."""
    if name is None:
        return None
    path = os.path.join(REPO, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        v = json.load(f).get(key)
    return None if v is None else round(float(v))


def make_inputs(cfg, indices, L, frames):
    """synthetic utterances by global index (prompt mel + text ids seeded by the index)."""
    mels, texts = [], []
    for i in indices:
        g = np.random.default_rng(2 + i)
        mels.append(torch.from_numpy(g.normal(-4.0, 2.0, (1, 100, frames)).astype(np.float32)))
        texts.append(torch.from_numpy(g.integers(2, int(cfg.gpt.number_text_tokens), L).astype(np.int64)))
    return mels, texts


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads():
    """threads for the CPU baseline: the cores this process may run on (sched affinity), capped by
    OMP_NUM_THREADS when the launcher sets it (the GPU box gives one GPU's job a 16-CPU share while
    os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    if os.environ.get("OMP_NUM_THREADS"):
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    return max(1, n)


def cpu_baseline(cfg, gsd, vsd, B, N, L, frames):
    """fp32 oracle (CPU restatement of the reference path, validated against the imported reference
    by tests/test_oracle_golden.py) on bounded samples, per phase: C2 shape (1 utterance) and a C3-shape
    sample (B utterances), N codes each (EOS suppressed).  ``value`` is the C3-shape sample's rate."""
    from indextts.gpt.conditioning import get_conditioning
    from indextts.vocoder.ecapa import speaker_embedding
    from oracle.bigvgan_oracle import BigVGANOracle, fold_weight_norm
    from oracle.gpt_oracle import GPTOracle
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    gt = {k: torch.from_numpy(np.asarray(v)) for k, v in gsd.items()}
    orc = GPTOracle(gt, cfg.gpt)
    voc = BigVGANOracle(vsd, cfg.bigvgan)
    vt = {k: v for k, v in fold_weight_norm(vsd).items()}

    def run(nb):
        mels, texts = make_inputs(cfg, range(nb), L, frames)
        ph = {}
        with torch.no_grad():
            t = time.perf_counter()
            mel = torch.cat(mels, 0)
            conds = get_conditioning(gt, cfg.gpt, mel)
            spk = speaker_embedding(vt, mel.transpose(1, 2))
            ph["conditioning_ecapa"] = time.perf_counter() - t
            t = time.perf_counter()
            codes = orc.generate(conds, torch.stack(texts), N, min_new_tokens=N)
            ph["decode"] = time.perf_counter() - t
            lat_t = voc_t = 0.0
            audio = 0.0
            for b in range(nb):
                t = time.perf_counter()
                fixed, _ = orc.remove_long_silence(codes[b:b + 1])
                lat = orc.latent(conds[b:b + 1], texts[b][None], fixed)
                lat_t += time.perf_counter() - t
                t = time.perf_counter()
                wav = voc.forward(lat, spk[b:b + 1])
                voc_t += time.perf_counter() - t
                audio += wav.shape[-1] / 24000.0
            ph["latent"], ph["vocoder"] = lat_t, voc_t
        tot = sum(ph.values())
        return audio, tot, {k: round(v, 3) for k, v in ph.items()}

    a2, t2, ph2 = run(1)
    # the C3-shape sample three times: the median is the value, min / max its spread (one run varied +-30 %
    # between boxes and calls)
    reps = [run(B) for _ in range(3)]
    rates = sorted(a / t for a, t, _ in reps)
    a3, t3, ph3 = sorted(reps, key=lambda r: r[0] / r[1])[1]
    return {"value": round(a3 / t3, 4), "unit": "audio-seconds/sec", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "visible_cpus": os.cpu_count(),
            "sample": f"C3-shape sample: {B} utterances x {N} codes (L={L}, {frames}-frame prompts, EOS suppressed), "
                      f"fp32 oracle incl. conditioning, ECAPA, greedy decode, latent pass and vocoder, run 3 times "
                      f"(median {a3:.2f} audio-s in {t3:.1f} s) on {threads} threads",
            "spread": {"min": round(rates[0], 4), "median": round(rates[1], 4), "max": round(rates[2], 4), "runs": 3},
            "phases_s": ph3, "c2": {"value": round(a2 / t2, 4), "sample": f"1 utterance x {N} codes", "phases_s": ph2}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--codes", type=int, default=400)
    ap.add_argument("--text-len", type=int, default=48)
    ap.add_argument("--prompt-frames", type=int, default=511)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--cpu-codes", type=int, default=96)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--breakdown", action="store_true", help="print per-phase times to stderr")
    ap.add_argument("--workload", choices=("c2", "c3", "c5"), default="c3",
                    help="BASELINE.json configs: c3 (default, the metric's config: batch 32 per GPU), c2 (one "
                         "utterance), c5 (srt_dubbing long-form: a synthetic SRT of --cues cues sharded over the "
                         "ranks, each rank's cue loop calling IndexTTS.infer per cue)")
    ap.add_argument("--cues", type=int, default=256)
    ap.add_argument("--c5-decoding", choices=("srt", "greedy"), default="srt",
                    help="C5: srt_dubbing's own decoding (the reference defaults its engine leaves in place) "
                         "or greedy")
    ap.add_argument("--decoding", choices=("greedy", "beam3"), default="greedy",
                    help="greedy (the headline) or beam3: the reference's default production decoding "
                         "(do_sample=True, num_beams=3, top_k=30, top_p=0.8, infer.py:535-543), 3 beam rows "
                         "per utterance (96-row decode step at batch 32)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group (RCCL) even at one rank, so the C4 gather of finished "
                         "int16 waveforms to rank 0 runs inside every timed step at N = 1 too")
    ap.add_argument("--pipeline", action="store_true",
                    help="run the K timed batches through BatchedTTS.synthesize_many (decode of batch i+1 "
                         "overlapped with the latent pass + vocoder of batch i)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ITTS_BENCH_DEVICE / ITTS_DIST_BACKEND=gloo: rehearse the N-rank path with several ranks on one GPU
    # (RCCL refuses two ranks on one device); the product setting is one rank per GPU over RCCL
    local = int(os.environ.get("ITTS_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or args.dist
    if use_dist:
        backend = os.environ.get("ITTS_DIST_BACKEND", "nccl")
        init = {} if world > 1 else dict(init_method=f"tcp://127.0.0.1:{os.environ.get('MASTER_PORT', '29511')}",
                                          world_size=1, rank=0)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, **init)
        else:
            dist.init_process_group(backend, **init)

    from indextts.pipeline import BatchedTTS, SR
    from indextts.sharding import gather_waveforms, shard
    from indextts.utils.config import default_config_path, load_config
    from indextts.utils.synthetic import bigvgan_state_dict, gpt_state_dict

    cfg = load_config(default_config_path())
    if args.workload == "c5":
        return long_form(args, cfg, dev, world, rank)
    gsd = gpt_state_dict(cfg.gpt, seed=0, mel_head_std=0.08)
    vsd = bigvgan_state_dict(cfg.bigvgan, seed=0)
    if args.workload == "c2":
        args.batch = 1
    B, N, L = args.batch, args.codes, args.text_len
    tts = BatchedTTS(gsd, vsd, cfg, dev, "bf16", max_kv=32 + L + 2 + 1 + N + 8)
    timer, t_act, t_amp, t_tail = KernelTimer(), KernelTimer(), KernelTimer(), KernelTimer()
    install_conv_timer(tts.vocoder, timer)
    install_hbm_timers(tts.vocoder, t_act, t_amp, t_tail)
    # global batch of B * world utterances; utterance i runs on rank i % world (weak scaling)
    mels, texts = make_inputs(cfg, shard(B * world, world, rank), L, args.prompt_frames)
    mels = [m.to(dev) for m in mels]
    texts = [t.to(dev) for t in texts]

    dec_kw = {}
    if args.decoding == "beam3":
        dec_kw = dict(do_sample=True, num_beams=3, top_k=30, top_p=0.8, temperature=1.0, seed=1234)

    def step():
        pcm, lens, _ = tts.synthesize(mels, texts, max_mel_tokens=N, min_new_tokens=N, **dec_kw)
        if use_dist:  # the one collective: finished int16 waveforms to rank 0, in utterance order
            gather_waveforms([pcm[b, : int(lens[b])] for b in range(B)], B * world, dev)
        return float(lens.sum()) / SR

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if not args.no_kernel_timing:
        tts.gpt.step_events = []  # HIP events around every decode-step graph replay
        if args.decoding == "beam3":  # distinct K/V rows per beam step (shared lineage counted once)
            tts.gpt.beam_lineage = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    audio = 0.0
    if args.pipeline:
        res = tts.synthesize_many([(mels, texts)] * args.steps, max_mel_tokens=N, min_new_tokens=N, **dec_kw)
        torch.cuda.synchronize()
        for pcm, lens, _ in res:
            if use_dist:
                gather_waveforms([pcm[b, : int(lens[b])] for b in range(B)], B * world, dev)
            audio += float(lens.sum()) / SR
    else:
        for _ in range(args.steps):
            audio += step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    step_ev, tts.gpt.step_events = tts.gpt.step_events, None
    if step_ev and tts.gpt.beam_lineage:  # beam3: distinct K/V rows per step, resolved after the timed region
        tts.gpt.beam_distinct_keys(step_ev, tts.gpt.beam_lineage)
    tts.gpt.beam_lineage = None
    if not args.no_kernel_timing:
        # the vocoder runs as ONE C-ABI call (itts_bigvgan_forward) in the timed steps; its implicit-GEMM
        # launches are timed one by one in an extra, untimed step through the Python launch sequence
        # (the same kernels, HipBigVGAN._forward_py)
        tts.vocoder.cforward = False
        timer.enabled = t_act.enabled = t_amp.enabled = t_tail.enabled = True
        step()
        torch.cuda.synchronize()
        timer.enabled = t_act.enabled = t_amp.enabled = t_tail.enabled = False
        tts.vocoder.cforward = True
    k_ms, k_flops, k_n = timer.result()
    dec = None
    if step_ev:
        d_ms = sum(a.elapsed_time(b) for a, b, _, _ in step_ev)
        d_bytes = sum(tts.gpt.step_weight_bytes + keys * tts.gpt.kv_bytes_per_key for _, _, _, keys in step_ev)
        gbs = d_bytes / (d_ms * 1e-3) / 1e9
        rows = step_ev[0][2]
        pl_st = {"B": rows, "kv_rows": True} if args.decoding == "beam3" else {"B": rows}
        pl = bool(tts.gpt.pl and tts.gpt._pl_ok(pl_st))
        body = ("20 x ONE persistent launch per layer (gpt_layer.hip: c_attn (ln_1 folded) -> attention -> "
                "attn.c_proj split-K 8 + reduce -> c_fc (ln_2 folded, gelu) -> mlp.c_proj split-K 8 + reduce as "
                "phases joined by in-launch hand-offs (epoch-tagged, nothing reset per step), weights prefetched "
                "by LDS-DMA) + last-layer reduce/ln_f/final_norm" if pl else
                "20 x [c_attn GEMM (ln_1 folded), attention, attn.c_proj GEMM split-K 8, reduce, c_fc GEMM "
                "(ln_2 folded, gelu), mlp.c_proj GEMM (split-K 8), reduce]")
        dec = {"kernel": f"GPT decode step, {rows} rows (hipGraph: {body} + mel_head GEMM + " +
                         ("beam candidates/select)" if args.decoding == "beam3" else "sampler)"), "bound": "hbm",
               "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
               "traffic": None, "launches": len(step_ev), "avg_launch_us": round(1e3 * d_ms / len(step_ev), 2),
               "algorithmic_bytes_per_launch": round(d_bytes / len(step_ev)), "share_of_step": round(d_ms / (1e3 * dt), 3)}
        if args.decoding == "beam3":
            dec["algorithmic_bytes_note"] = ("weights + distinct K/V rows per step: each utterance's prompt once, "
                                             "generated positions once per distinct cache row among its beams "
                                             "(lineage table at each replay's end), the step's new keys")
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
        a = torch.tensor([audio], device=dev, dtype=torch.float64)
        dist.all_reduce(a, op=dist.ReduceOp.SUM)
        audio = float(a)
    if rank != 0:
        dist.destroy_process_group()
        return
    achieved = (k_flops / (k_ms * 1e-3) / 1e12) if k_ms > 0 else None
    voc = {"kernel": "itts_igemm_fwd (BigVGAN convs C >= 192 and ConvTranspose phases, MFMA bf16)", "bound": "mfma",
           "achieved": None if achieved is None else round(achieved, 2), "peak": PEAK_BF16_TFLOPS,
           "unit": "TFLOP/s", "frac": None if achieved is None else round(achieved / PEAK_BF16_TFLOPS, 4),
           "traffic": _traffic(TRAFFIC_VOCODER.get(args.workload), "igemm_bytes_per_launch"), "launches": k_n,
           "avg_launch_us": round(1e3 * k_ms / max(k_n, 1), 2),
           "algorithmic_bytes_per_launch": round(timer.bytes / max(k_n, 1)),
           "share_of_step": round(k_ms / (1e3 * dt / args.steps), 3)}
    hbm = {}
    for key, t, name, tkey in (("roofline_vocoder_act", t_act, "itts_aa_snakebeta_fwd (Activation1d, every AMP "
                                "stage)", "aa_snakebeta_bytes_per_launch"),
                               ("roofline_vocoder_amp", t_amp, "itts_amp_conv_fwd (AMPBlock1 dilated convs "
                                "+ residuals, C = 24 / 48 / 96)", "amp_conv_bytes_per_launch"),
                               ("roofline_vocoder_tail", t_tail, "itts_act_conv_post_tanh (activation_post + "
                                "conv_post + tanh + int16 in one launch)", "act_post_conv_bytes_per_launch")):
        ms, _, n = t.result()
        if n:
            gbs = t.bytes / (ms * 1e-3) / 1e9
            hbm[key] = {"kernel": name, "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": _traffic(TRAFFIC_VOCODER.get(args.workload), tkey),
                        "launches": n, "avg_launch_us": round(1e3 * ms / n, 2),
                        "algorithmic_bytes_per_launch": round(t.bytes / n),
                        "share_of_step": round(ms / (1e3 * dt / args.steps), 3)}
    if dec is not None:  # the decode step: the dominant unit of work
        tf = TRAFFIC_DECODE.get((args.workload, args.decoding, pl))
        dec["traffic"] = None if tf is None else _traffic(tf, "bytes_per_step")
        dec["traffic_source"] = None if tf is None else f"profiles/{tf}"
    cpu = None
    if args.breakdown:
        ph = {}
        step_t = tts.synthesize(mels, texts, max_mel_tokens=N, min_new_tokens=N, timings=ph)
        print("breakdown (s):", json.dumps({k: round(v, 4) for k, v in ph.items()}), file=sys.stderr, flush=True)
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(cfg, gsd, vsd, args.cpu_batch, args.cpu_codes, L, args.prompt_frames)
    out = {
        "metric": METRIC, "value": round(audio / dt, 3), "unit": "audio-seconds/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic: seeded random-init IndexTTS-1.5 weights, random 511-frame prompt mels, random text ids",
        # the driver's contract: value = the whole-job aggregate over all ranks (the metric's "/GPU" is
        # per_gpu_value; at N = 1 they coincide)
        "value_is": "whole-job aggregate over all GPUs; per_gpu_value = value / n_gpus",
        "per_gpu_value": round(audio / dt / world, 3),
        "decoding": "greedy" if args.decoding == "greedy" else "beam sample, num_beams=3, top_k=30, top_p=0.8",
        "config": {"workload": f"{'C2' if args.workload == 'c2' else 'C3'}: batch={B} zero-shot utterance"
                               f"{'s' if B > 1 else ''} per GPU (one prompt each), L={L} text ids, "
                               f"{N} codes each (EOS suppressed): conditioning+ECAPA, GPT prefill+decode (hipGraph), "
                               "latent pass, BigVGAN2 -> int16" + (", pipelined batches" if args.pipeline else ""),
                   "global_batch": B * world, "seq_len": N, "parallelism": f"dp{world}",
                   "collective": (f"{dist.get_backend()} gather of finished int16 waveforms to rank 0 in every "
                                  "timed step") if use_dist else None},
        "roofline": dec,
        "roofline_vocoder_conv": voc,
        **hbm,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


WORDS = ("mind the gap please stand clear of closing doors there is a vehicle arriving in dock next station "
         "last stop change here for northern line thank you travelling with us take all your belongings "
         "this train terminates platform passengers are reminded to keep their luggage with them").split()


def synthetic_srt(tokenizer, n_cues, seed=3):
    """C5's synthetic SRT: n_cues cue texts of L ~ U[8, 96] BPE tokens each (seeded words)."""
    g = np.random.default_rng(seed)
    texts = []
    for L in g.integers(8, 97, n_cues):
        words = []
        while len(tokenizer.tokenize(" ".join(words))) < L:
            words.append(WORDS[int(g.integers(len(WORDS)))])
        texts.append(" ".join(words).capitalize() + ".")
    return texts


def _write_prompt_wav(path, seconds=5.0, sr=24000, seed=3):
    import wave
    g = np.random.default_rng(seed)
    t = np.arange(int(seconds * sr)) / sr
    sig = 0.3 * np.sin(2 * np.pi * (140 + 60 * np.sin(2 * np.pi * 0.7 * t)) * t) + 0.03 * g.standard_normal(t.size)
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes((sig * 32767).astype("<i2").tobytes())


class _Cue:  # srt_parser.SRTEntry's fields the strategies read
    def __init__(self, index, text):
        self.index, self.text, self.duration = index, text, 0.0


def long_form(args, cfg, dev, world, rank):
    """C5 (BASELINE.json configs[4]): srt_dubbing long-form THROUGH THE DROP-IN API.  A synthetic SRT of
    args.cues cues (L ~ U[8, 96] tokens, seed 3) and one prompt wav; a synthetic IndexTTS-1.5
    checkpoint directory in the reference's layout (seeded weights) loaded by ``IndexTTS(cfg_path,
    model_dir, is_fp16=True)`` as srt_dubbing's IndexTTSEngine builds it; per rank, cue i (i % world ==
    rank) is synthesised by BasicStrategy's loop -- ``for i, entry in enumerate(entries):
    infer(text=entry.text, audio_prompt=voice, output_path=None, **filtered)``
    (srt_dubbing/src/strategies/basic_strategy.py:65-74, tts_engines/index_tts_engine.py:45-63).  The
    cue lookahead batches the loop (chunks of LONGFORM_BATCH rows; with ITTS_DEVICES a single process
    deals them over several GPUs); the finished int16 waveforms are gathered to rank 0 over RCCL.
    --c5-decoding srt: srt_dubbing's decoding = the reference defaults (IndexTTSEngine's
    inspect.signature filter drops every decoding kwarg, Q9: beam sample, num_beams 3, top_k 30,
    top_p 0.8, max_mel_tokens 600); greedy: do_sample=False, num_beams=1.  One step = the whole SRT."""
    import tempfile
    from indextts.infer import IndexTTS
    from indextts.pipeline import SR
    from indextts.sharding import gather_waveforms, shard
    from indextts.utils.synthetic import write_checkpoint_dir
    root = os.environ.get("ITTS_BENCH_CKPT") or os.path.join(tempfile.gettempdir(), "itts_bench_ckpt")
    if rank == 0:
        write_checkpoint_dir(root, cfg, os.path.join(REPO, "tests", "golden", "tiny_bpe.model"), seed=0,
                             mel_head_std=0.08)
        _write_prompt_wav(os.path.join(root, "voice.wav"))
    if world > 1:
        dist.barrier()
    voice = os.path.join(root, "voice.wav")
    tts = IndexTTS(cfg_path=os.path.join(root, "config.yaml"), model_dir=root, is_fp16=True, device=str(dev))
    texts = synthetic_srt(tts.tokenizer, args.cues)
    mine = shard(len(texts), world, rank)
    entries = [_Cue(i + 1, texts[i]) for i in mine]
    kw = {} if args.c5_decoding == "srt" else dict(do_sample=False, num_beams=1)

    def step():
        pcm = []
        for i, entry in enumerate(entries):  # BasicStrategy.process_entries (engine filters kwargs: Q9)
            _, data = tts.infer(text=entry.text, audio_prompt=voice, output_path=None, **kw)
            pcm.append(torch.from_numpy(data.reshape(-1)))
        audio = sum(float(p.numel()) for p in pcm) / SR
        if world > 1:  # in this rank's shard order
            gather_waveforms([p.to(dev) for p in pcm], len(texts), dev)
        return audio

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    audio = 0.0
    for _ in range(args.steps):
        audio += step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
        a = torch.tensor([audio], device=dev, dtype=torch.float64)
        dist.all_reduce(a, op=dist.ReduceOp.SUM)
        audio = float(a)
    ndev = tts.n_devices
    tts.close()
    if rank == 0:
        dec = ("srt_dubbing's decoding (reference defaults: beam sample, num_beams=3, top_k=30, top_p=0.8, "
               "max_mel_tokens=600)" if args.c5_decoding == "srt" else "greedy, max_mel_tokens=600")
        print(json.dumps({
            "metric": METRIC, "value": round(audio / dt, 3), "unit": "audio-seconds/sec", "n_gpus": world * ndev,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
            "value_is": "whole-job aggregate over all GPUs; per_gpu_value = value / n_gpus",
            "per_gpu_value": round(audio / dt / (world * ndev), 3), "audio_seconds": round(audio / args.steps, 2),
            "data": "synthetic: seeded random-init IndexTTS-1.5 checkpoint directory, one 5 s prompt wav, "
                    "synthetic SRT cue texts (tiny BPE)",
            "decoding": dec,
            "config": {"workload": f"C5: srt long-form, {len(texts)} cues (L ~ U[8,96] tokens) through "
                                   f"IndexTTS.infer per cue (BasicStrategy loop; cue lookahead batching, "
                                   f"chunks of {IndexTTS.LONGFORM_BATCH} rows), sharded over {world} rank(s) x "
                                   f"{ndev} device(s) per rank, RCCL gather",
                       "global_batch": len(texts), "seq_len": None, "parallelism": f"dp{world * ndev}"}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
