"""The C-ABI boundary: libitts_hip.so loads (no GPU needed) and exports exactly the entry points
declared in include/itts_hip.h, and the ctypes table in indextts/_hip.py binds the same set with
the same arity.  No compute calls here (CPU suite)."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "itts_hip.h")


def header_decls():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decls = {}
    for m in re.finditer(r"^(?:const\s+)?\w+\s*\*?\s*(itts_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.M):
        args = m.group(2).strip()
        decls[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return decls


@pytest.fixture(scope="module")
def lib():
    from indextts import _build, _hip
    _build.build(verbose=False)  # no-op when up to date
    return _hip.load()


def test_header_parses():
    d = header_decls()
    assert len(d) >= 17 and "itts_aa_snakebeta_bct" in d and "itts_decode_gemm" in d


def test_library_exports_every_header_symbol(lib):
    for name in header_decls():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (itts_\w+)", out))
    assert exported == set(header_decls()), exported ^ set(header_decls())


def test_ctypes_table_matches_header():
    from indextts import _hip
    decl = header_decls()
    assert set(_hip.SIGNATURES) == set(decl)
    for name, (_, argtypes) in _hip.SIGNATURES.items():
        assert len(argtypes) == decl[name], name


def test_runtime_queries(lib):
    assert lib.itts_abi_version() == 5
    assert lib.itts_build_target() == b"gfx950"


def test_argument_errors_do_not_launch(lib):
    """Argument validation happens before any HIP call, so it is observable without a GPU."""
    from indextts import _hip
    rc = lib.itts_igemm_pack_dims(0, 8, None, None)
    assert rc != 0 and b"bad args" in lib.itts_last_error()
    ci, co = ctypes.c_int32(), ctypes.c_int32()
    assert lib.itts_igemm_pack_dims(100, 100, ctypes.byref(ci), ctypes.byref(co)) == 0
    assert (ci.value, co.value) == (128, 128)  # K chunk 32 (Cin < 128), N tile 32 (Cout < 128)
    rc = lib.itts_decode_gemm(None, 0, None, 24, 32, 1, None, None, None, None, None, 0, 0, 0, None, 0, 0, 0, 1, None)
    assert rc != 0 and b"bad sizes" in lib.itts_last_error()
    with pytest.raises(_hip.HipError):
        _hip.check(rc, "itts_decode_gemm")


def test_product_path_fails_loudly_without_library(tmp_path, monkeypatch):
    import importlib
    from indextts import _hip
    monkeypatch.setattr(_hip, "_lib", None)
    with pytest.raises(_hip.HipError, match="no CPU fallback"):
        _hip.load(str(tmp_path / "missing.so"))
    importlib.reload(_hip)


def test_step_struct_layouts_match(lib):
    """ctypes mirrors of ItTsGptLayerW / ItTsGptWeights / ItTsGptDecodeState / ItTsSampling have the
    C sizes (field order is the ABI), and the state-size query answers without a GPU."""
    from indextts import _hip
    for i, c in enumerate((_hip.GptLayerW, _hip.GptWeights, _hip.GptDecodeState, _hip.Sampling, _hip.Conv, _hip.Act,
                           _hip.AmpLayer, _hip.BigvganStage, _hip.BigvganWeights, _hip.GptSeqLayerW,
                           _hip.GptSeqWeights, _hip.GptPlLayerW)):
        assert lib.itts_struct_size(i) == ctypes.sizeof(c), c.__name__
    assert lib.itts_struct_size(99) == -1
    w = _hip.GptWeights(2, 256, 4, 8194, 8208, 8192, 8193)
    sizes = (ctypes.c_int64 * _hip.GPT_STATE_NBUF)()
    assert lib.itts_gpt_decode_state_bytes(ctypes.byref(w), 5, 64, 16, sizes) == 0
    D, R, Rp = 256, 5, 32
    assert list(sizes)[:7] == [R * D * 4, Rp * D * 2, R * 3 * D * 4, Rp * D * 2, Rp * 4 * D * 2, 8 * R * D * 4,
                               R * 8208 * 4]
    assert sizes[7] == sizes[8] == 2 * R * 4 * 64 * 64 * 2
    assert lib.itts_gpt_decode_state_bytes(ctypes.byref(w), 0, 64, 16, sizes) != 0
