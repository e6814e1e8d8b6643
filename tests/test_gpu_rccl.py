"""The C4 collective on the GPU: ``gather_waveforms`` (indextts/sharding.py) over RCCL (torch's
"nccl" backend on ROCm) with device int16 rows of ragged lengths.  World size 1 on the one-GPU box
(the 8-rank node run is the driver's); it exercises the exact calls bench.py makes at N > 1 --
``all_gather`` of the int64 lengths, ``gather`` of the uint8 payload to rank 0 -- on HBM buffers,
and checks the order and every byte.  There is no reference counterpart: the reference has no
inference-side collective."""
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_gather_waveforms_world1_device_rows():
    from indextts.sharding import gather_waveforms
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", world_size=1, rank=0,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        g = torch.Generator(device=dev).manual_seed(4)
        lens = [1024 * k + r for k, r in ((3, 0), (17, 5), (1, 1023), (400, 0), (0, 7), (9, 2))]
        rows = [torch.randint(-32767, 32768, (n,), generator=g, device=dev, dtype=torch.int32).to(torch.int16)
                for n in lens]
        out = gather_waveforms(rows, len(rows), dev)
        torch.cuda.synchronize()
        assert out is not None and len(out) == len(rows)
        for src, got in zip(rows, out):
            assert got.device.type == "cuda" and got.dtype == torch.int16
            assert torch.equal(got, src)
    finally:
        dist.destroy_process_group()
