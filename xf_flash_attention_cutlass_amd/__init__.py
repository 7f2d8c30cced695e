"""xf_flash_attention_cutlass_amd — MI355X-native (gfx950) flash attention.

Drop-in for Sherlolo/xf_flash_attention_cutlass's hot path:
  * C ABI   : lib/libpaged-attention.so   (include/paged_attn.h; csrc/paged_attn.h of the ref)
  * pybind  : module `paged_attn`          (fwd / varlen_fwd / fwd_kvcache / bwd / varlen_bwd;
                                             export.cpp of the ref)
  * Python  : flash_attn_func, flash_attn_varlen_func, flash_attn_with_kvcache
                                            (test.py:41-245 of the ref), with autograd.

The native libraries are required: importing this package on a machine where they were not
built raises ImportError (there is no CPU or eager fallback).
"""
from __future__ import annotations

import importlib.util
import os
import sysconfig

import torch  # noqa: F401  (must be imported first: it provides libamdhip64 / libtorch_hip)

_HERE = os.path.dirname(os.path.abspath(__file__))
_EXT = os.path.join(_HERE, "lib", "paged_attn" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def _load_paged_attn():
    if not os.path.exists(_EXT):
        raise ImportError(f"native module {_EXT} is missing: run `python "
                          "xf_flash_attention_cutlass_amd/build.py` or "
                          "`python __graft_entry__.py build` (no fallback exists)")
    spec = importlib.util.spec_from_file_location("paged_attn", _EXT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


paged_attn = _load_paged_attn()

from .interface import (  # noqa: E402
    flash_attn_fp8_func,
    flash_attn_func,
    flash_attn_kvpacked_func,
    flash_attn_varlen_func,
    flash_attn_varlen_kvpacked_func,
    flash_attn_with_kvcache,
)

__all__ = [
    "paged_attn",
    "flash_attn_func",
    "flash_attn_fp8_func",
    "flash_attn_kvpacked_func",
    "flash_attn_varlen_func",
    "flash_attn_varlen_kvpacked_func",
    "flash_attn_with_kvcache",
]
