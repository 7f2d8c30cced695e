"""CPU: the C-ABI library loads, exports every symbol include/paged_attn.h declares, and its
host-side validation reports errors through fmha_last_error() instead of throwing/exiting
(reference behaviour was exit(-1)/C++ exceptions across extern "C", flash_hip.h:21-42).
No kernel is launched here."""
import ctypes
import os
import re
import subprocess

import pytest

from xf_flash_attention_cutlass_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "paged_attn.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(fmha_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_reference_entry_points():
    syms = header_symbols()
    for ref_sym in ("fmha_fwd", "fmha_varlen_fwd", "fmha_page_kvcache_fwd"):
        assert ref_sym in syms


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", capi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (\w+)$", out, flags=re.M))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    assert set(capi.EXPORTED) == set(header_symbols())


def test_library_has_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={capi.LIB_PATH}"], capture_output=True, text=True)
    blob = open(capi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_header_compiles_as_c():
    r = subprocess.run(["gcc", "-x", "c", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__",
                        "-I/opt/rocm/include", "-I", os.path.dirname(HEADER), "-"],
                       input='#include "paged_attn.h"\nint main(void){return 0;}\n', text=True,
                       capture_output=True)
    assert r.returncode == 0, r.stderr


def test_version():
    assert capi.lib().fmha_version().decode().startswith("xf-fmha-gfx950")


def _fwd(**over):
    a = dict(q=16, k=16, v=16, o=16, alibi=None, sq=16, sk=16, b=1, h=4, hk=2, d=64, p=0.0,
             stream=None, dprops=None, scale=0.125, p_ptr=None, lse=None, wl=-1, wr=-1,
             softcap=0.0, ret=False, fp16=False, splits=1)
    a.update(over)
    L = capi.lib()
    L.fmha_fwd(*a.values())
    return L.fmha_last_status(), L.fmha_last_error().decode()


@pytest.mark.parametrize("over,needle", [
    (dict(q=None), "non-null"),
    (dict(b=0), "batch size"),
    (dict(h=3, hk=2), "must divide"),
    (dict(d=60), "multiple of 8"),
    (dict(d=512), "at most 256"),
    (dict(p=1.0), "p_dropout"),
    (dict(p=-0.1), "p_dropout"),
    (dict(ret=True), "return_softmax"),
    (dict(p=0.1, ret=True), "p and softmax_lse"),
    (dict(sk=0), "positive"),
])
def test_fwd_validation_errors(over, needle):
    status, msg = _fwd(**over)
    assert status != 0 and needle in msg


def test_error_state_is_cleared_by_next_call():
    status, _ = _fwd(b=0)
    assert status != 0
    L = capi.lib()
    L.fmha_page_kvcache_fwd(16, 16, 16, None, None, 16, None, None, 64, 1, 64, 1, 4, 4, 64, 16,
                            None, 0.125, -1, -1, 1, None, None, None, False, False, False)
    # missing block table is a validation error, reported with a new message
    assert L.fmha_last_status() != 0 and "block_table" in L.fmha_last_error().decode()


def test_error_is_thread_local():
    import threading
    _fwd(b=0)
    seen = {}

    def other():
        seen["status"] = capi.lib().fmha_last_status()
    th = threading.Thread(target=other)
    th.start(); th.join()
    assert seen["status"] == 0


def test_pybind_module_surface():
    import xf_flash_attention_cutlass_amd as xfa
    for op in ("fwd", "varlen_fwd", "fwd_kvcache", "bwd", "varlen_bwd"):
        assert hasattr(xfa.paged_attn, op)
