"""Several GPUs behind ONE unchanged ``IndexTTS`` (BASELINE.json configs[4]).

srt_dubbing is a single process that calls ``IndexTTS.infer`` once per cue
(``srt_dubbing/src/strategies/basic_strategy.py:65-74`` -> ``tts_engines/index_tts_engine.py:45-63``).
With ``ITTS_DEVICES`` set (``"0,1,2,3"``, or ``"all"`` for every visible GPU) the ``IndexTTS`` built by
that caller owns one worker process per listed device besides its own engine: each is a fresh
``spawn``-ed child (fork + exec of a new interpreter, never a fork of the GPU-initialised parent)
that builds its own ``IndexTTS`` on its GPU and answers ``infer_many`` requests over a pipe.  The
cue lookahead (``IndexTTS.prefetch``) deals the upcoming cues over the parent's engine and the
workers (longest first onto the least-loaded device), waits for every share and files the results
per cue, so ``infer`` returns each cue's PCM in the caller's order exactly as before.  Rows never
interact inside the batched pipeline, so a cue's int16 PCM does not depend on which device or batch
produced it (deterministic decoding: bit for bit; ``tests/test_gpu_longform.py::
test_two_engines_one_gpu_equal_per_call`` checks it with two processes on ONE GPU and short rows).

A worker that does not answer within ``ITTS_WORKER_TIMEOUT`` seconds (default 600 per request,
1800 to load), or answers out of step (a reply for another request id), is terminated and marked
dead; the caller redoes its share locally (``IndexTTS._infer_many_devices``).

Utterances shard with no data-path collective: what crosses processes is the finished int16 PCM
(pickled through the pipe), as the north star's "only a gather of finished waveforms".  The
torchrun form of the same data parallelism (one rank per GPU, RCCL gather) is ``indextts.sharding``.
"""
from __future__ import annotations

import itertools
import multiprocessing as mp
import os
import traceback
from typing import Dict, List, Optional, Sequence, Tuple


def parse_devices(spec: Optional[str], n_visible: int) -> List[str]:
    """``ITTS_DEVICES`` -> device strings ("cuda:i"); "" / None -> []; "all" -> every visible GPU.
    Entries may repeat (two workers on one GPU: the tests' stand-in for two GPUs)."""
    if not spec:
        return []
    spec = spec.strip()
    if spec == "all":
        return [f"cuda:{i}" for i in range(n_visible)]
    out = []
    for tok in spec.split(","):
        tok = tok.strip()
        if not tok:
            continue
        i = int(tok[5:] if tok.startswith("cuda:") else tok)
        if not 0 <= i < max(n_visible, 1):
            raise ValueError(f"ITTS_DEVICES entry {tok!r}: only {n_visible} GPU(s) visible")
        out.append(f"cuda:{i}")
    return out


def _load_builder(spec: str):
    mod, _, name = spec.partition(":")
    import importlib
    return getattr(importlib.import_module(mod), name)


def _worker_main(conn, cfg_path: str, model_dir: str, is_fp16: bool, device: str,
                 builder: str = "indextts.infer:IndexTTS", no_pl: bool = False):
    """Child process: its own IndexTTS on ``device``; serves (rid, prompt, texts, max_tokens, gen).
    ``builder`` ("module:callable", the IndexTTS class by default) lets the CPU tests run the
    protocol with a stand-in engine.  ``no_pl``: the device is shared with another engine, so the
    persistent decode layer (which needs the whole GPU resident) is off (ITTS_PL=0)."""
    os.environ["ITTS_DEVICES"] = ""  # no nested pools
    if no_pl:
        os.environ["ITTS_PL"] = "0"
    try:
        tts = _load_builder(builder)(cfg_path=cfg_path, model_dir=model_dir, is_fp16=is_fp16, device=device)
        tts.LOOKAHEAD = 0
    except BaseException:  # noqa: BLE001 -- reported to the parent, which then runs without this worker
        conn.send(("init", "error", traceback.format_exc()))
        conn.close()
        return
    conn.send(("init", "ok", device))
    while True:
        try:
            msg = conn.recv()
        except EOFError:
            break
        if msg is None:
            break
        rid, prompt, texts, max_tokens, gen = msg
        try:
            res = tts.infer_many(prompt, texts, None, False, max_tokens, **gen)
            conn.send((rid, "ok", [(int(sr), data) for sr, data in res]))
        except BaseException:  # noqa: BLE001
            conn.send((rid, "error", traceback.format_exc()))
    conn.close()


class WorkerError(RuntimeError):
    pass


class DevicePool:
    """Worker processes, one per device entry, each with its own IndexTTS (lazy readiness: the
    workers load their weights while the parent builds its own engine)."""

    def __init__(self, cfg_path: str, model_dir: str, is_fp16: bool, devices: Sequence[str],
                 builder: str = "indextts.infer:IndexTTS", no_pl=()):
        ctx = mp.get_context("spawn")
        self.devices = list(devices)
        self.request_timeout = float(os.environ.get("ITTS_WORKER_TIMEOUT", "600"))
        self.init_timeout = max(self.request_timeout, 1800.0)
        self._conns, self._procs, self._ready = [], [], []
        self._rid = itertools.count()
        for d in self.devices:
            parent, child = ctx.Pipe(duplex=True)
            p = ctx.Process(target=_worker_main, args=(child, cfg_path, model_dir, bool(is_fp16), d, builder,
                                                       d in no_pl),
                            daemon=True, name=f"itts-worker-{d}")
            p.start()
            child.close()
            self._conns.append(parent)
            self._procs.append(p)
            self._ready.append(None)  # None: not yet confirmed; True: serving; False: dead

    def __len__(self):
        return len(self.devices)

    def _kill(self, i: int):
        """Mark worker i dead and stop its process (a hung or out-of-step worker is never reused)."""
        self._ready[i] = False
        p = self._procs[i]
        if p.is_alive():
            p.terminate()
            p.join(timeout=10)

    def _recv(self, i: int, timeout: float):
        """conn.recv() bounded by ``timeout`` seconds; a timeout kills the worker."""
        conn = self._conns[i]
        if not conn.poll(timeout):
            self._kill(i)
            raise WorkerError(f"worker {self.devices[i]}: no reply within {timeout:.0f} s")
        return conn.recv()

    def _wait_ready(self, i: int) -> bool:
        if self._ready[i] is None:
            try:
                tag, status, info = self._recv(i, self.init_timeout)
                self._ready[i] = tag == "init" and status == "ok"
                if not self._ready[i]:
                    print(f">> IndexTTS worker on {self.devices[i]} failed to start:\n{info}")
                    self._kill(i)
            except (EOFError, OSError, WorkerError):
                self._kill(i)
        return bool(self._ready[i])

    def alive(self) -> List[int]:
        return [i for i in range(len(self.devices)) if self._wait_ready(i)]

    def submit(self, i: int, prompt, texts: List[str], max_tokens: int, gen: dict) -> Tuple[int, int]:
        rid = next(self._rid)
        try:
            self._conns[i].send((rid, prompt, list(texts), int(max_tokens), dict(gen)))
        except (OSError, BrokenPipeError) as e:
            self._ready[i] = False
            raise WorkerError(f"worker {self.devices[i]}: {e}") from e
        return i, rid

    def result(self, ticket: Tuple[int, int]):
        i, rid = ticket
        try:
            got, status, payload = self._recv(i, self.request_timeout)
        except (EOFError, OSError) as e:
            self._kill(i)
            raise WorkerError(f"worker {self.devices[i]} died: {e}") from e
        if got != rid:  # the pipe is out of step (e.g. an interrupted earlier request): never reuse it
            self._kill(i)
            raise WorkerError(f"worker {self.devices[i]}: reply {got} for request {rid}")
        if status != "ok":
            raise WorkerError(f"worker {self.devices[i]}: {payload}")
        return payload

    def close(self):
        for c in self._conns:
            try:
                c.send(None)
            except (OSError, BrokenPipeError):
                pass
        for p in self._procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
        for c in self._conns:
            c.close()
        self._conns, self._procs, self._ready = [], [], []


def deal(costs: Sequence[int], n_bins: int) -> List[List[int]]:
    """Longest-processing-time assignment: item indices per bin, each bin's items in input order."""
    load = [0] * n_bins
    bins: List[List[int]] = [[] for _ in range(n_bins)]
    for i in sorted(range(len(costs)), key=lambda k: (-costs[k], k)):
        b = min(range(n_bins), key=lambda j: (load[j], j))
        bins[b].append(i)
        load[b] += max(int(costs[i]), 1)
    return [sorted(b) for b in bins]
