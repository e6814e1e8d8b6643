"""Multi-process (gloo, world_size 2, CPU) test of the data-parallel utterance sharding and the
rank-0 waveform gather used by bench.py --gpus N."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wave(i):
    g = torch.Generator().manual_seed(1000 + i)
    n = 1024 * (3 + (i * 7) % 11)  # ragged lengths, whole frames
    return torch.randint(-32767, 32767, (n,), generator=g, dtype=torch.int32).to(torch.int16)


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from indextts.sharding import gather_waveforms, shard
        rows = [_wave(i) for i in shard(n_total, world, rank)]
        out = gather_waveforms(rows, n_total)
        if rank == 0:
            ok = all(torch.equal(out[i], _wave(i)) for i in range(n_total))
            q.put(("ok" if ok else "mismatch", [int(o.numel()) for o in out]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 7), (2, 2), (2, 1), (3, 10)])
def test_gather_waveforms_in_utterance_order(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, lens = q.get(timeout=10)
    assert status == "ok"
    assert lens == [_wave(i).numel() for i in range(n_total)]


def test_shard_is_a_partition():
    from indextts.sharding import shard
    for world in (1, 2, 3, 8):
        for n in (0, 1, 5, 32, 256):
            got = sorted(i for r in range(world) for i in shard(n, world, r))
            assert got == list(range(n))
