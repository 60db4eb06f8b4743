"""ctypes binding of libsmer_hip.so (the C-ABI declared in include/smer_hip.h).

The library is loaded after `import torch` so that it binds the same HIP
runtime (libamdhip64.so.7) that PyTorch-ROCm already mapped.  There is no
fallback: if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be imported before the HIP library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SMER_HIP_LIB") or os.path.join(_HERE, "libsmer_hip.so")

c_int, c_long, c_float, c_size, c_u32 = (ctypes.c_int, ctypes.c_long, ctypes.c_float,
                                         ctypes.c_size_t, ctypes.c_uint32)
P = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/smer_hip.h
SIGNATURES = {
    "smer_abi_version": (c_int, []),
    "smer_last_error": (ctypes.c_char_p, []),
    "smer_gemm": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P,
                          c_float, c_int, P, c_long, P, c_long, c_float, c_float, c_u32, P,
                          c_long, P, c_long, c_int, P, c_size, P]),
    "smer_gemm_debug_stamps": (c_int, [P, c_size]),
    "smer_gemm_wgrad_bias": (c_int, [c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_long,
                                     c_int, P, c_int, P, c_size, P]),
    "smer_embed_fwd_fp8": (c_int, [c_int, c_int, P, P, c_int, P, P, c_float, c_float, c_u32, P, c_long, P, c_long,
                                   P, P, P]),
    "smer_gemm_wgrad_fp8": (c_int, [c_int, c_int, c_int, P, c_long, P, c_long, P, P, P, c_long, c_int, P, c_int,
                                    P, c_size, c_int, P]),
    "smer_gemm_wgrad_bias_ex": (c_int, [c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_long,
                                        c_int, P, c_int, P, c_size, c_int, P]),
    "smer_attn_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P,
                              c_long, P, c_long, P, P, c_int, c_float, c_float, c_u32, P, c_int, P]),
    "smer_attn_fwd_fp8": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_long,
                                  P, c_long, P, P, c_int, c_float, c_float, c_u32, P, c_int, P, c_long,
                                  P, P, P]),
    "smer_attn_drop_mask_gen": (c_int, [c_int, c_int, c_int, c_int, c_float, c_u32, P, P]),
    "smer_attn_drop_mask_bytes": (c_size, [c_int, c_int, c_int, c_int]),
    "smer_attn_bwd_workspace": (c_size, [c_int, c_int, c_int, c_int, c_int]),
    "smer_attn_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P,
                              c_long, P, c_long, P, c_long, P, P, c_int, c_float, c_float, c_u32,
                              P, c_long, P, c_long, P, c_long, P, c_size, P, P]),
    "smer_attn_bwd_fp8": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_long,
                                  P, c_long, P, c_long, P, P, c_int, c_float, c_float, c_u32, P, c_long,
                                  P, c_long, P, c_long, P, c_size, P, P, c_long, P, c_long, P, c_long,
                                  P, P, P]),
    "smer_attn_weights": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long,
                                  P, P, c_int, c_float, P, P]),
    "smer_attn_decode": (c_int, [c_int, c_int, c_int, c_int, P, c_long, P, P, c_long, c_long,
                                 c_long, P, P, P, c_long, c_float, P]),
    "smer_attn_decode_qln": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_float, P, c_long, P,
                                     P, c_long, c_int, P, P, c_long, c_long, c_long, P, P, P, c_long,
                                     c_float, P]),
    "smer_kv_scatter_heads": (c_int, [c_int, c_int, c_int, c_int, P, c_long, P, c_long, c_long,
                                      c_long, P, P, P]),
    "smer_kv_scatter": (c_int, [c_int, c_int, c_int, P, c_long, P, c_long, c_long, P, P, P]),
    "smer_linear_decode": (c_int, [c_int, c_int, c_int, P, c_long, P, c_long, P, c_int, P, c_long,
                                   P, c_long, P, c_long, P, c_long, c_long, P, P, c_int, P]),
    "smer_linear_decode_ln": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_float, P, c_long, P,
                                      c_long, P, c_int, P, c_long, P, c_long, P, c_long, P, c_long,
                                      c_long, P, P, c_int, P]),
    "smer_linear_decode_f32": (c_int, [c_int, c_int, c_int, P, c_long, P, c_long, P, c_int, P, c_long,
                                       P, c_long, P, c_long, P, c_long, c_long, P, P, c_int, P]),
    "smer_linear_decode_ln_f32": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_float, P, c_long, P,
                                          c_long, P, c_int, P, c_long, P, c_long, P, c_long, P, c_long,
                                          c_long, P, P, c_int, P]),
    "smer_attn_decode_split_f32": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_long, c_long, c_long, P, P, P,
                                           c_float, P]),
    "smer_attn_decode_split_qln_f32": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_float, P, c_long, P, P,
                                               c_long, c_int, P, P, c_long, c_long, c_long, P, P, P, c_float, P]),
    "smer_linear_decode_merge_f32": (c_int, [c_int, c_int, c_int, P, P, c_long, P, c_int, P, c_long, P, c_long, P,
                                             c_long, P]),
    "smer_fp8_quantize_workspace": (c_size, []),
    "smer_fp8_quantize": (c_int, [c_int, c_int, P, c_long, P, c_long, P, P, P]),
    "smer_fp8_quantize_segments": (c_int, [c_int, P, P, P, c_int, P]),
    "smer_gemm_fp8": (c_int, [c_int, c_int, c_int, P, c_long, P, c_long, P, P, P, c_int, P, c_long,
                              c_float, c_u32, P, c_long, P]),
    "smer_gemm_fp8_q": (c_int, [c_int, c_int, c_int, P, c_long, P, c_long, P, P, P, c_int, P,
                                c_long, c_float, c_u32, P, c_long, P, c_long, P, P, P]),
    "smer_layernorm_fwd_fp8": (c_int, [c_int, c_int, P, c_long, P, P, c_float, P, c_long, P, P, P,
                                       c_long, P, P, P]),
    "smer_fp8_scales": (c_int, [c_int, P, P, P, P, P]),
    "smer_fp8_quantize_segments_t": (c_int, [c_int, P, P, P, c_int, P]),
    "smer_gemm_fp8_ex": (c_int, [c_int, c_int, c_int, P, c_long, P, c_long, P, P, P, c_int, P, c_long,
                                 P, c_long, c_float, c_float, c_u32, P, c_long, P, c_long, P, P, P]),
    "smer_gemm_fp8_gate8": (c_int, [c_int, c_int, c_int, P, c_long, P, c_long, P, P, P, c_long, c_float,
                                    P, c_long, P, c_long, P, P, P]),
    "smer_layernorm_bwd_fp8": (c_int, [c_int, c_int, P, c_long, P, c_long, P, P, P, P, c_long, P, c_long,
                                       c_float, c_u32, P, c_long, P, P, P, P, c_int, P, c_size, c_int,
                                       P]),
    "smer_grammar_greedy_step": (c_int, [c_int, c_int, P, c_long, P, c_int, P, c_int, P, P, c_int,
                                         c_int, c_int, c_int, P, P, P, P, c_int, P, P]),
    "smer_grammar_greedy_step_ring": (c_int, [c_int, c_int, P, c_long, P, c_int, P, c_int, P, P,
                                              c_int, c_int, c_int, c_int, P, P, P, P, c_int, P, P,
                                              c_int, P]),
    "smer_grammar_sample_step": (c_int, [c_int, c_int, P, c_long, P, c_int, P, c_int, P, P, P,
                                         c_int, c_int, c_int, c_int, P, P, P, P, c_int, P, P, P,
                                         c_int, P]),
    "smer_layernorm_fwd": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_float, P, c_long, P,
                                   P, P]),
    "smer_layernorm_bwd_workspace": (c_size, [c_int, c_int]),
    "smer_layernorm_bwd": (c_int, [c_int, c_int, c_int, P, c_long, c_int, P, c_long, P, P, P, P,
                                   c_long, P, c_long, c_float, c_u32, P, P, c_int, P, c_size, P]),
    "smer_layernorm_bwd_partials": (c_int, [c_int, c_int, c_int, P, c_long, c_int, P, c_long, P, P,
                                            P, P, c_long, P, c_long, c_float, c_u32, P, c_size, P]),
    "smer_layernorm_param_reduce": (c_int, [c_int, c_int, P, c_size, P, P, c_int, P]),
    "smer_embed_fwd": (c_int, [c_int, c_int, c_int, P, P, c_int, P, P, c_float, c_float, c_u32,
                               P, c_long, P]),
    "smer_embed_bwd_workspace": (c_size, [c_int, c_int, c_int]),
    "smer_embed_bwd": (c_int, [c_int, c_int, c_int, c_float, P, P, c_long, c_int, c_float, c_u32,
                               P, P, c_long, c_int, c_float, c_u32, P, P, c_size, P]),
    "smer_wce_denom": (c_int, [c_int, P, P, P, P]),
    "smer_wce_fwd_bwd": (c_int, [c_int, c_int, c_int, P, c_long, P, P, P, P, P, P, c_long,
                                 c_float, P]),
    "smer_adam": (c_int, [c_long, P, P, P, P, P, c_float, c_float, c_float, c_float, c_float,
                          c_float, P]),
    "smer_cast": (c_int, [c_int, c_int, c_long, P, P, P]),
    "smer_cast2d": (c_int, [c_int, c_int, c_int, c_int, P, c_long, P, c_long, P]),
    "smer_colsum_workspace": (c_size, [c_int, c_int]),
    "smer_colsum": (c_int, [c_int, c_int, c_int, P, c_long, P, c_int, P, c_size, P]),
    "smer_debug_checksum": (c_int, [P, c_long, c_long, c_long, P, c_int, P]),
    "smer_argmax_accuracy": (c_int, [c_int, c_int, P, c_long, P, P, c_int, c_int, P, P]),
}

_lib = None
_load_error = None


def load():
    """Load (once) and return the ctypes library; raise if unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        _load_error = "libsmer_hip.so not built (%s); run __graft_entry__.build()" % LIB_PATH
        raise RuntimeError(_load_error)
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class SmerError(RuntimeError):
    pass


def check(status, what):
    if status != 0:
        msg = load().smer_last_error()
        raise SmerError("%s failed (%d): %s" % (what, status, msg.decode() if msg else ""))


def call(name, *args):
    lib = load()
    check(getattr(lib, name)(*args), name)
