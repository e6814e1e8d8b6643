"""Data-parallel sharding of utterances across GPUs.

One process per GPU; utterance i is synthesised on rank ``i % world`` (independent units, no
cross-rank state besides the replicated weights and per-prompt caches); the only collective is the
final gather of finished int16 waveforms to rank 0, in the original utterance order:
``all_gather`` of the per-rank lengths, then one ``gather`` of each rank's concatenated PCM padded
to the largest rank payload.  Backend-agnostic: RCCL (``"nccl"``) with device tensors on MI355X,
``gloo`` with CPU tensors in the tests.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


def shard(n_items: int, world: int, rank: int) -> List[int]:
    """indices of the utterances owned by ``rank`` (round-robin)."""
    return list(range(rank, n_items, world))


def gather_waveforms(rows: List[torch.Tensor], n_total: int, device=None) -> Optional[List[torch.Tensor]]:
    """rows: this rank's int16 waveforms, for the indices ``shard(n_total, world, rank)`` in order.
    -> on rank 0 the ``n_total`` waveforms in utterance order; None on other ranks."""
    world, rank = dist.get_world_size(), dist.get_rank()
    device = torch.device(device) if device is not None else (rows[0].device if rows else torch.device("cpu"))
    if dist.get_backend() == "gloo":  # gloo collectives run on host buffers
        device = torch.device("cpu")
    per = (n_total + world - 1) // world  # max utterances per rank
    mine = shard(n_total, world, rank)
    assert len(rows) == len(mine), (len(rows), len(mine))
    lens = torch.zeros(per, dtype=torch.int64, device=device)
    for j, r in enumerate(rows):
        lens[j] = r.numel()
    all_lens = [torch.zeros_like(lens) for _ in range(world)]
    dist.all_gather(all_lens, lens)
    cap = max(int(x.sum()) for x in all_lens)
    buf = torch.zeros(max(cap, 1), dtype=torch.int16, device=device)
    if rows:
        flat = torch.cat([r.reshape(-1).to(device, torch.int16) for r in rows])
        buf[: flat.numel()] = flat
    # int16 is not reducible by every backend's gather; ship the bytes
    payload = buf.view(torch.uint8)
    bufs = [torch.empty_like(payload) for _ in range(world)] if rank == 0 else None
    dist.gather(payload, bufs, dst=0)
    if rank != 0:
        return None
    out: List[Optional[torch.Tensor]] = [None] * n_total
    for r in range(world):
        pcm = bufs[r].view(torch.int16)
        off = 0
        for j, idx in enumerate(shard(n_total, world, r)):
            n = int(all_lens[r][j])
            out[idx] = pcm[off: off + n]
            off += n
    return out
