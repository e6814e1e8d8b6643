"""ctypes binding of libitts_hip.so -- the C-ABI boundary of the HIP hot path (include/itts_hip.h).

The library is built in-tree (``indextts/_build.py``; ``__graft_entry__.build()``) for gfx950 and
loaded AFTER ``import torch`` so it binds torch's already-loaded ``libamdhip64.so.7`` (same soname
as ROCm 7.2's), i.e. one HIP runtime per process.  There is no fallback: if the library is missing
or a call fails, a ``RuntimeError`` is raised (the reference's loader silently fell back to torch,
``indextts/infer.py:97-109``; here the HIP path is the product).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported first: provides the HIP runtime)

LIB_NAME = "libitts_hip.so"
_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG_DIR, LIB_NAME)

F32, BF16, F16 = 0, 1, 2

_c_i = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_f = ctypes.c_float
_vp = ctypes.c_void_p
_i32p = ctypes.POINTER(ctypes.c_int32)

# name -> (restype, argtypes); keep in sync with include/itts_hip.h
SIGNATURES = {
    "itts_last_error": (ctypes.c_char_p, []),
    "itts_abi_version": (_c_i, []),
    "itts_build_target": (ctypes.c_char_p, []),
    "itts_struct_size": (_c_i64, [_c_i]),
    "itts_aa_snakebeta_fwd": (_c_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_i, _c_i, _c_i, _c_i64, _c_i64, _c_i64,
                                     _c_i64, _c_i64, _c_i64, _c_i, _c_i, _vp]),
    "itts_aa_snakebeta_bct": (_c_i, [_vp, _vp, _vp, _vp, _vp, _vp, _c_i, _c_i, _c_i, _c_i, _vp]),
    "itts_igemm_pack_dims": (_c_i, [_c_i, _c_i, _i32p, _i32p]),
    "itts_igemm_fwd": (_c_i, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _c_i, _c_i,
                              _c_i, _c_i, _c_i, _i32p, _c_i, _c_i, _c_f, _c_i, _c_i, _vp]),
    "itts_amp_conv_fwd": (_c_i, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp,
                                 _c_i, _c_i, _c_i, _c_i, _c_i, _i32p, _c_f, _vp]),
    "itts_conv_post_tanh":(_c_i, [_vp, _c_i64, _c_i64, _vp, _c_f, _c_i, _c_i, _vp, _c_i, _c_i, _vp, _vp, _c_i64,
                                   _c_i, _vp]),
    "itts_act_conv_post_tanh": (_c_i, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_f, _c_i, _c_i, _vp, _c_i, _c_i,
                                       _vp, _vp, _c_i64, _vp]),
    "itts_log_mel": (_c_i, [_vp, _c_i64, _c_i, _c_i, _vp, _vp, _c_i, _c_i, _c_i, _vp, _vp]),
    "itts_resample_sinc": (_c_i, [_vp, _c_i64, _c_i, _c_i, _vp, _c_i, _c_i, _c_i, _vp, _c_i64, _c_i, _vp]),
    "itts_igemm_splitk": (_c_i, [_vp, _c_i64, _c_i, _c_i, _vp, _c_i, _c_i, _vp, _vp, _vp, _vp]),
    "itts_pad_rows_bf16": (_c_i, [_vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, _c_i, _c_i, _c_i, _c_i, _c_i, _c_i, _vp,
                                  _vp]),
    "itts_relu_affine_rows": (_c_i, [_vp, _c_i64, _c_i64, _c_i, _c_i, _c_i, _vp, _vp, _vp, _c_i64, _c_i64, _vp]),
    "itts_time_stats": (_c_i, [_vp, _c_i64, _c_i64, _vp, _c_i64, _c_i64, _c_i, _c_i, _c_i, _c_f, _vp, _vp, _vp]),
    "itts_cond_rel_attn": (_c_i, [_vp, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _c_i, _c_i, _c_i, _c_f, _vp, _c_i64, _c_i,
                                  _vp]),
    "itts_cross_attn": (_c_i, [_vp, _c_i64, _c_i64, _vp, _vp, _c_i64, _c_i64, _vp, _c_i, _c_i, _c_i, _c_i, _c_f, _vp,
                               _c_i64, _c_i64, _vp]),
    "itts_cond_subsample": (_c_i, [_vp, _c_i64, _c_i64, _c_i, _c_i, _c_i, _vp, _vp, _c_i, _vp, _vp]),
    "itts_cond_glu_dwconv": (_c_i, [_vp, _c_i64, _c_i, _c_i, _c_i, _vp, _vp, _c_i, _vp, _vp, _c_f, _vp, _c_i64, _vp,
                                    _vp]),
    "itts_layernorm_rows": (_c_i, [_vp, _c_i64, _vp, _vp, _c_i64, _c_i, _c_i, _vp, _vp, _vp, _vp, _c_i, _vp]),
    "itts_residual_reduce_ln": (_c_i, [_vp, _c_i64, _vp, _c_i, _c_i64, _c_i64, _vp, _vp, _c_i64, _c_i, _c_i, _vp, _vp,
                                       _vp, _vp, _c_i, _vp]),
    "itts_gemm_f32": (_c_i, [_vp, _c_i64, _vp, _c_i64, _c_i, _c_i, _c_i, _vp, _c_i, _vp, _vp, _c_i64, _vp]),
    "itts_attn_decode": (_c_i, [_vp, _c_i64, _c_i, _c_i64, _vp, _vp, _vp, _c_i64, _c_i64, _c_i, _vp, _c_i, _vp, _vp,
                                _c_i64, _c_i, _c_i,
                                _c_i, _c_i, _vp]),
    "itts_attn_decode_rows": (_c_i, [_vp, _c_i64, _c_i, _c_i64, _vp, _vp, _vp, _c_i64, _c_i64, _c_i, _vp, _c_i, _vp,
                                     _vp, _c_i64, _c_i, _c_i, _c_i, _c_i, _vp, _c_i64, _vp]),
    "itts_attn_decode_proj": (_c_i, [_vp, _c_i64, _c_i, _c_i64, _vp, _vp, _vp, _c_i64, _c_i64, _c_i, _vp, _c_i, _vp,
                                     _vp, _c_i, _vp, _c_i64, _c_i64, _c_i, _c_i, _c_i, _vp, _c_i64, _vp]),
    "itts_decode_gemm16": (_c_i, [_vp, _c_i64, _vp, _c_i, _c_i, _c_i, _vp, _c_i, _vp, _c_i64, _c_i, _vp]),
    "itts_decode_gemm16x": (_c_i, [_vp, _c_i64, _vp, _c_i, _c_i, _c_i, _vp, _vp, _c_f, _c_i, _c_i, _vp, _c_i64, _c_i,
                                   _vp, _c_i64, _c_i, _vp]),
    "itts_beam_candidates": (_c_i, [_vp, _c_i64, _c_i, _vp, _vp, _vp, _c_i, _c_i, _c_i, _c_f, _c_i, _c_f, _c_i, _c_f,
                                    _c_i, _vp, _vp, _vp, _c_i, _vp]),
    "itts_beam_select": (_c_i, [_vp, _vp, _vp, _c_i, _c_i, _c_i, _c_i, _c_f, _vp, _c_i, _vp, _vp, _vp, _c_i64, _vp,
                                _c_i64, _vp, _c_i, _vp, _c_i64, _c_i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_i,
                                _c_i, _vp, _vp, _vp, _vp, _c_i, _c_i, _c_i, _vp]),
    "itts_attn_prefill": (_c_i, [_vp, _c_i64, _vp, _vp, _vp, _c_i, _c_i, _vp, _vp, _c_i64, _c_i64, _vp, _c_i64, _c_i,
                                 _c_i, _c_i, _vp]),
    "itts_sample_embed": (_c_i, [_vp, _c_i64, _c_i, _vp, _vp, _vp, _c_i64, _vp, _c_i, _c_i, _c_i, _c_f, _vp, _vp, _c_i,
                                 _c_i, _vp, _vp, _vp, _vp, _c_i, _c_i, _vp, _vp]),
    "itts_sample_topk_embed": (_c_i, [_vp, _c_i64, _c_i, _vp, _vp, _vp, _c_i64, _vp, _c_i, _c_i, _c_i, _c_f, _c_f,
                                      _c_i, _c_f, _vp, _vp, _c_i, _c_i, _vp, _vp, _vp, _vp, _c_i, _c_i, _vp, _vp]),
    "itts_step_advance": (_c_i, [_vp, _c_i, _vp]),
    "itts_decode_gemm": (_c_i, [_vp, _c_i64, _vp, _c_i, _c_i, _c_i, _vp, _vp, _vp, _vp, _vp, _c_i, _c_i, _c_i, _vp,
                                _c_i64, _c_i, _c_i64, _c_i, _vp]),
    "itts_gpt_forward_rows_workspace_bytes": (_c_i64, [_vp, _c_i64]),
    "itts_gpt_forward_rows": (_c_i, [_vp, _vp, _c_i64, _vp, _vp, _vp, _c_i, _c_i, _vp, _vp, _c_i64, _c_i64, _c_i64,
                                     _c_i, _vp, _c_i, _vp, _c_i, _vp, _vp]),
    "itts_gpt_prefill": (_c_i, [_vp, _vp, _vp, _vp, _c_i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "itts_gpt_decode_state_bytes": (_c_i, [_vp, _c_i, _c_i, _c_i, _vp]),
    "itts_gpt_fold_ln": (_c_i, [_vp, _vp, _vp, _vp, _c_i, _c_i, _vp, _vp, _vp]),
    "itts_gpt_pack_frag": (_c_i, [_vp, _c_i, _c_i, _c_i, _c_i, _vp]),
    "itts_gpt_pack_qkv12": (_c_i, [_vp, _vp, _vp, _c_i, _c_i, _vp, _vp]),
    "itts_gpt_decode_step": (_c_i, [_vp, _vp, _vp, _vp]),
    "itts_gpt_decode_steps": (_c_i, [_vp, _vp, _vp, _c_i, _vp]),
    "itts_gpt_pl_scratch_bytes": (_c_i64, []),
    "itts_gpt_pl_supported": (_c_i, [_vp, _c_i]),
    "itts_gpt_pl_reset": (_c_i, [_vp, _vp]),
    "itts_gpt_layer_pl": (_c_i, [_vp, _vp, _vp, _c_i, _c_i, _c_i, _vp, _vp]),
    "itts_gpt_pl_error": (_c_i, [_vp, _vp, ctypes.POINTER(_c_i)]),
    "itts_gpt_decode_steps_pl": (_c_i, [_vp, _vp, _vp, _vp, _vp, _c_i, _vp]),
    "itts_bigvgan_workspace_bytes": (_c_i64, [_vp, _c_i, _c_i]),
    "itts_bigvgan_forward": (_c_i, [_vp, _vp, _vp, _vp, _c_i, _c_i, _vp, _vp, _vp, _vp]),
    "itts_diag_occupy": (_c_i, [_c_i, _c_i, _vp, _vp]),
}


GPT_STATE_NBUF = 14  # itts_gpt_decode_state_bytes() entries

# ---- structs of the whole-step entry point (include/itts_hip.h; field order is the ABI) ----------
class GptLayerW(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("qkv_w16", "qkv_u", "qkv_c", "o_w16", "o_c", "fc_w16", "fc_u", "fc_c",
                                   "proj_w", "proj_b", "o_w")]


class GptPlLayerW(ctypes.Structure):
    _fields_ = [("qkv_w12", _vp), ("qkv_uc", _vp)]


class GptWeights(ctypes.Structure):
    _fields_ = [("n_layer", _c_i), ("d_model", _c_i), ("n_head", _c_i), ("n_mel_codes", _c_i),
                ("logits_pitch", _c_i), ("start_mel", _c_i), ("stop_mel", _c_i),
                ("layers", ctypes.POINTER(GptLayerW))] + \
        [(n, _vp) for n in ("ln_f_g", "ln_f_b", "final_g", "final_b", "head_w", "head_b", "mel_emb", "mel_pos")]


class GptDecodeState(ctypes.Structure):
    _fields_ = [("rows", _c_i), ("max_kv", _c_i), ("kv_base", _c_i), ("max_new", _c_i)] + \
        [(n, _vp) for n in ("x", "xh", "qkv", "o", "f", "part", "logits", "k_cache", "v_cache", "pad", "tstate",
                            "kv_rows")] + \
        [("ld_rows", _c_i64)] + [(n, _vp) for n in ("seen", "done", "codes", "forced")] + [("num_beams", _c_i)]


class GptSeqLayerW(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("qkv_w", "o_w", "fc_w", "proj_w", "qkv_b", "o_b", "fc_b", "proj_b", "ln1_g",
                                   "ln1_b", "ln2_g", "ln2_b")]


class GptSeqWeights(ctypes.Structure):
    _fields_ = [("n_layer", _c_i), ("d_model", _c_i), ("n_head", _c_i), ("dtype", _c_i),
                ("layers", ctypes.POINTER(GptSeqLayerW))] + \
        [(n, _vp) for n in ("ln_f_g", "ln_f_b", "final_g", "final_b", "head_w_f32")]


class Sampling(ctypes.Structure):
    _fields_ = [("mode", _c_i), ("min_new", _c_i), ("rep_penalty", _c_f), ("temperature", _c_f), ("top_k", _c_i),
                ("top_p", _c_f)]

_lib = None
_lock = threading.Lock()


class HipError(RuntimeError):
    pass


def load(path: str = None):
    """Load (once) and return the ctypes library; raises if it is absent or incomplete."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("ITTS_HIP_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise HipError(f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                           "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)  # AttributeError = stale library
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def exported_symbols():
    return list(SIGNATURES)


def check(rc: int, name: str):
    if rc != 0:
        msg = _lib.itts_last_error().decode(errors="replace") if _lib else ""
        raise HipError(f"{name} failed (rc={rc}): {msg}")


def ptr(t) -> int:
    """Device pointer of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(t) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float16:
        return F16
    raise HipError(f"unsupported dtype {t.dtype}")


def i32_array(vals):
    arr = (ctypes.c_int32 * len(vals))(*[int(v) for v in vals])
    return arr


# ---- structs of the whole-vocoder entry point (include/itts_hip.h) --------------------------------
class Conv(ctypes.Structure):
    _fields_ = [("w", _vp), ("bias", _vp), ("cin", _c_i), ("cout", _c_i), ("ntaps", _c_i),
                ("tap_off", ctypes.c_int32 * 16)]


class Act(ctypes.Structure):
    _fields_ = [("up12", _vp), ("down12", _vp), ("log_alpha", _vp), ("log_beta", _vp)]


class AmpLayer(ctypes.Structure):
    _fields_ = [("a1", Act), ("c1", Conv), ("a2", Act), ("c2", Conv)]


class BigvganStage(ctypes.Structure):
    _fields_ = [("up_rate", _c_i), ("phases", ctypes.POINTER(Conv)), ("cond_w", _vp), ("cond_b", _vp),
                ("n_blocks", _c_i), ("n_layers", _c_i), ("layers", ctypes.POINTER(AmpLayer)), ("amp_mode", _c_i)]


class BigvganWeights(ctypes.Structure):
    _fields_ = [("n_stages", _c_i), ("gpt_dim", _c_i), ("spk_dim", _c_i), ("conv_pre", Conv), ("cond_pre_w", _vp),
                ("cond_pre_b", _vp), ("stages", ctypes.POINTER(BigvganStage)), ("act_post", Act), ("post_w", _vp),
                ("post_b", _c_f), ("post_k", _c_i)]
