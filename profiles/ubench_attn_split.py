"""Decode attention (EXPERIMENT, kernel removed after measurement; it lives in commit 1e046aa): one workgroup per (head, row) (itts_attn_decode) vs split-S chunks with a
last-arriver merge (itts_attn_decode_split), B = 32 rows, bf16 K/V from HBM (rotating caches),
hipGraph back-to-back launches.  Also checks the split result against the unsplit one and its
run-to-run bit identity.  Library from ITTS_HIP_LIB (variant builds: ITTS_ASPLIT_NT / _KB)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "index-tts-dubbing_amd"), os.path.join(REPO, "profiles")]
import torch  # noqa: E402
from indextts import _hip  # noqa: E402
from ubench_decode import graph_time, lib  # noqa: E402

_vp, _i, _i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lib.itts_attn_decode_split.argtypes = [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i, _vp, _i, _vp, _vp, _i64, _i, _i, _i,
                                       _i, _vp, _i64, _vp, _vp, _i, _vp]
lib.itts_attn_split_params.argtypes = [_vp, _vp]
nt, kb = ctypes.c_int(), ctypes.c_int()
per_round = lib.itts_attn_split_params(ctypes.byref(nt), ctypes.byref(kb))
tag = os.environ.get("TAG", "")
D, H, Smax, NKV = 1024, 16, 600, 6
ws = torch.zeros(128 * H * 8 * 72, device="cuda")
cnt = torch.zeros(128 * H, dtype=torch.int32, device="cuda")
for B, S in ((32, 283), (32, 142), (32, 460), (96, 283)):
    kcs = [torch.randn(B, H, Smax, 64, device="cuda").to(torch.bfloat16) for _ in range(NKV)]
    vcs = [torch.randn(B, H, Smax, 64, device="cuda").to(torch.bfloat16) for _ in range(NKV)]
    qkv = torch.randn(B * 3 * D, device="cuda")
    o = torch.zeros(max(B, 32), D, dtype=torch.bfloat16, device="cuda")
    o2 = torch.zeros_like(o)
    pad = torch.zeros(B, dtype=torch.int32, device="cuda")
    kvb = min(82, S - 2)
    t = torch.tensor([S - 1 - kvb, 0, 0, 0], dtype=torch.int32, device="cuda")

    def fa(i, out=o):
        _hip.check(lib.itts_attn_decode(qkv.data_ptr(), 3 * D, 1, B * 3 * D, None, kcs[i % NKV].data_ptr(),
                                        vcs[i % NKV].data_ptr(), kcs[0].stride(0), kcs[0].stride(1), Smax,
                                        pad.data_ptr(), kvb, t.data_ptr(), out.data_ptr(), D, B, H, 1, 1,
                                        _hip.stream_ptr()), "attn")
    base = graph_time(fa)
    fa(0)
    ref = o.clone()
    line = f"[{tag} NT={nt.value} KB={kb.value}] B={B} S={S}: unsplit {base:.2f} us ({B * H * S * 256 / base / 1e3:.0f} GB/s)"
    for rounds in (1, 2, 3):
        chunk = per_round * rounds
        if (Smax + chunk - 1) // chunk > 8 or chunk >= 2 * S:
            continue

        def fs(i, out=o2, chunk=chunk):
            _hip.check(lib.itts_attn_decode_split(qkv.data_ptr(), 3 * D, None, kcs[i % NKV].data_ptr(),
                                                  vcs[i % NKV].data_ptr(), kcs[0].stride(0), kcs[0].stride(1), Smax,
                                                  pad.data_ptr(), kvb, t.data_ptr(), out.data_ptr(), D, B, H, 1, 1,
                                                  None, 0, ws.data_ptr(), cnt.data_ptr(), chunk, _hip.stream_ptr()),
                       "split")
        ts = graph_time(fs)
        fs(0)
        a = o2.clone()
        fs(0)
        same = bool(torch.equal(a, o2))
        err = float((a.float() - ref.float()).abs().max())
        line += f" | chunk {chunk}: {ts:.2f} us ({B * H * S * 256 / ts / 1e3:.0f} GB/s) maxdiff {err:.1e} repro {same}"
    print(line, flush=True)
    del kcs, vcs
