"""ctypes binding of libpaged-attention.so (the C ABI in include/paged_attn.h).

This is the same binding a maintainer would add on the reference side to call the C ABI
without torch types (INTEGRATION.md shows it).  Tensors are passed as raw device pointers;
the current torch stream is passed as the hipStream_t.  No fallback: if the native library
is missing this module raises at import.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libpaged-attention.so")
# the same C ABI with the non-default kernels compiled in (build.py: XFA_VARIANTS=1), for A/B
# runs and the bit-identity tests only
VARIANTS_PATH = os.path.join(_HERE, "lib", "variants", "libpaged-attention.so")

vp, i32, f32, b_, sz = C.c_void_p, C.c_int32, C.c_float, C.c_bool, C.c_size_t

_SIGS = {
    "fmha_fwd": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, vp, vp, f32, vp, vp,
                 C.c_int, C.c_int, f32, b_, b_, C.c_int],
    "fmha_varlen_fwd": [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, f32, b_, b_,
                        C.c_int, C.c_int],
    "fmha_page_kvcache_fwd": [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32,
                              i32, vp, f32, C.c_int, C.c_int, i32, vp, vp, vp, b_, b_, b_],
    "fmha_fwd_strided": [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32,
                         C.POINTER(C.c_int64), f32, C.c_int, C.c_int, f32, b_, C.c_int, vp,
                         f32, vp],
    "fmha_fwd_fp8": [vp, vp, vp, vp, vp, f32, f32, f32, i32, i32, i32, i32, i32, i32, f32,
                     C.c_int, C.c_int, b_, vp],
    "fmha_varlen_fwd_ex_v2": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, i32, i32, i32, i32,
                           i32, i32, i32, i32, f32, C.c_int, C.c_int, f32, b_, vp, f32, vp],
    "fmha_page_kvcache_fwd_ex_v2": [vp, vp, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, i32, i32,
                                 i32, f32, C.c_int, C.c_int, f32, vp, i32, i32, i32, f32, f32, vp,
                                 b_, vp],
    "fmha_bwd": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32,
                 f32, C.c_int, C.c_int, f32, b_, b_, vp, vp, sz],
    "fmha_bwd_workspace_size_v2": [i32, i32, i32, i32, i32, i32, b_],
    "fmha_varlen_bwd_v2": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32,
                        i32, i32, i32, i32, f32, C.c_int, C.c_int, f32, b_, b_, vp, vp, sz, vp,
                        f32],
    "fmha_varlen_bwd_workspace_size_v2": [i32, i32, i32, i32, i32, i32, b_],
    "fmha_kvcache_append": [vp, vp, vp, vp, vp, vp, i32, vp, i32, i32, vp, vp, vp, vp, i32, b_,
                            b_, i32, i32, i32, i32, i32, b_, vp],
    "fmha_last_error": [],
    "fmha_last_status": [],
    "fmha_last_num_splits": [],
    "fmha_last_kernel": [],
    "fmha_version": [],
    "fmha_set_rng_state": [C.c_uint64, C.c_uint64],
    "fmha_set_rng_state_device": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p],
    "fmha_set_option": [C.c_char_p, C.c_int],
    "fmha_get_option": [C.c_char_p],
}
_RES = {"fmha_last_error": C.c_char_p, "fmha_last_kernel": C.c_char_p, "fmha_version": C.c_char_p, "fmha_last_status": C.c_int,
        "fmha_last_num_splits": C.c_int,
        "fmha_set_option": C.c_int, "fmha_get_option": C.c_int,
        "fmha_bwd_workspace_size_v2": sz, "fmha_varlen_bwd_workspace_size_v2": sz}

EXPORTED = tuple(_SIGS)


def load(path: str = LIB_PATH, strict: bool = True) -> C.CDLL:
    """Load a build of the library; strict=False tolerates symbols an older build (an A/B
    variant, tools/lib_ab.py) does not export."""
    if not os.path.exists(path):
        raise ImportError(f"native library {path} is missing: run `python "
                          "xf_flash_attention_cutlass_amd/build.py` (no CPU fallback exists)")
    lib = C.CDLL(path)
    for name, args in _SIGS.items():
        plain = name[:-3] if name.endswith("_v2") else None
        if not hasattr(lib, name):
            if strict:
                getattr(lib, name)                 # raises: the build lacks a declared symbol
            if not (plain and hasattr(lib, plain)):
                continue
            name = plain                           # an older (2.0) A/B build: plain names
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RES.get(name, _RES.get(name + "_v2"))
        if plain:
            setattr(lib, plain, fn)                # the header's macro names, as C callers see them
    return lib


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = load()
    return _lib


class FmhaError(RuntimeError):
    pass


def check() -> None:
    """Raise the thread-local error of the last call, if any (mirrors TORCH_CHECK)."""
    L = lib()
    if L.fmha_last_status() != 0:
        raise FmhaError(L.fmha_last_error().decode())


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
