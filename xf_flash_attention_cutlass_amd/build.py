"""Build the gfx950 native code in-tree (no cmake/ninja needed for the C ABI).

Produces
  xf_flash_attention_cutlass_amd/lib/libpaged-attention.so   — the C-ABI library
      (include/paged_attn.h; replaces the reference's CMake target `paged-attention`,
      CMakeLists.txt:29-33), hipcc --offload-arch=gfx950, no torch dependency;
  xf_flash_attention_cutlass_amd/lib/paged_attn*.so          — the pybind/ATen module
      `paged_attn` (export.cpp equivalent), linked against libpaged-attention.so.

  xf_flash_attention_cutlass_amd/lib/variants/libpaged-attention.so — the same C ABI built with
      XFA_VARIANTS=1: also the kernels no default path runs (the 4-wave D = 128 forward, fwd_w4
      = 1; the ping-pong fp8 forward, fp8_w4 = 2), for A/B runs and the bit-identity tests
      (tests/test_kernel_variants_gpu.py); the product library refuses those option values.

Usage: python xf_flash_attention_cutlass_amd/build.py [--no-ext] [--no-variants] [-j N] [--force]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
OBJ = os.path.join(PKG, "lib", "obj")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("XFA_ARCH", "gfx950")
LIBNAME = "libpaged-attention.so"

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-I", CSRC, "-I", INCLUDE]
# extra -D/-f flags for A/B variants of the library (tools/build_variant.sh); not for releases
HIP_FLAGS += os.environ.get("XFA_EXTRA_FLAGS", "").split()

VARIANTS = [(hd, dt) for hd in (64, 128, 256) for dt in ("bf16", "f16")]
BWD_HDS = (64, 128, 256)     # backward head-dim buckets (as the forward)


def _newer(out: str, deps) -> bool:
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in deps)


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def _compile(job):
    src, out, defs = job
    deps = [src, __file__] + _headers()
    if _newer(out, deps):
        return out, None
    cmd = [HIPCC, *HIP_FLAGS, *defs, "-c", src, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return out, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return out, None


VARIANT_TUS = {"fmha_fwd_hd128_bf16.o", "fmha_fwd_hd128_f16.o", "fmha_fwd_fp8.o", "fmha_api.o"}
VARIANTS_DIR = os.path.join(LIB, "variants")


def build_lib(jobs: int = 8, force: bool = False, verbose: bool = False, variants: bool = False) -> str:
    """variants: lib/variants/libpaged-attention.so; the translation units XFA_VARIANTS changes
    are rebuilt with it (into lib/obj_variants), the others shared with the product build."""
    obj_dir = os.path.join(LIB, "obj_variants") if variants else OBJ
    os.makedirs(obj_dir, exist_ok=True)
    todo = []
    for hd, dt in VARIANTS:
        defs = [f"-DXFA_HD={hd}", f"-DXFA_DTN={dt}", f"-DXFA_DT_BF16={1 if dt == 'bf16' else 0}"]
        for kind in (("fwd", "bwd") if hd in BWD_HDS else ("fwd",)):
            src = os.path.join(CSRC, f"fmha_{kind}.hip")
            todo.append((src, os.path.join(OBJ, f"fmha_{kind}_hd{hd}_{dt}.o"), defs))
    todo.append((os.path.join(CSRC, "fmha_append.hip"), os.path.join(OBJ, "fmha_append.o"), []))
    todo.append((os.path.join(CSRC, "fmha_fwd_fp8.hip"), os.path.join(OBJ, "fmha_fwd_fp8.o"), []))
    todo.append((os.path.join(CSRC, "fmha_api.cpp"), os.path.join(OBJ, "fmha_api.o"), []))
    if variants:
        todo = [(src, os.path.join(obj_dir, os.path.basename(out)), defs + ["-DXFA_VARIANTS=1"])
                for src, out, defs in todo if os.path.basename(out) in VARIANT_TUS]
        todo += [(None, os.path.join(OBJ, n), None) for n in sorted(os.listdir(OBJ))
                 if n.endswith(".o") and n not in VARIANT_TUS]
    if force:
        for src, out, _ in todo:
            if src and os.path.exists(out):
                os.remove(out)
    errors = []
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for out, err in ex.map(_compile, [t for t in todo if t[0]]):
            if err:
                errors.append(err)
            elif verbose:
                print("built", os.path.relpath(out, ROOT))
    if errors:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errors))
    objs = [o for _, o, _ in todo]
    if variants:
        os.makedirs(VARIANTS_DIR, exist_ok=True)
    so = os.path.join(VARIANTS_DIR if variants else LIB, LIBNAME)
    soname = "libpaged-attention-variants.so" if variants else LIBNAME
    if not _newer(so, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so, *objs,
               "-Wl,-soname," + soname]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return so


def build_c_smoke(force: bool = False) -> str:
    """tests/bin/c_smoke: the torch-free C++ caller of the C ABI (tests/c_smoke.cpp), linked only
    against libpaged-attention.so (rpath to the in-tree lib/)."""
    src = os.path.join(ROOT, "tests", "c_smoke.cpp")
    out_dir = os.path.join(ROOT, "tests", "bin")
    out = os.path.join(out_dir, "c_smoke")
    so = os.path.join(LIB, LIBNAME)
    if not os.path.exists(src):
        return ""
    if not force and _newer(out, [src, so, os.path.join(INCLUDE, "paged_attn.h")]):
        return out
    os.makedirs(out_dir, exist_ok=True)
    cmd = [HIPCC, "-O2", "-std=c++17", f"--offload-arch={ARCH}", "-I", INCLUDE, src, "-o", out,
           f"-L{LIB}", "-l:" + LIBNAME, "-Wl,-rpath,$ORIGIN/../../xf_flash_attention_cutlass_amd/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"c_smoke build failed:\n$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return out


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(LIB, "paged_attn" + suffix)


def build_ext(force: bool = False, verbose: bool = False) -> str:
    """pybind11/ATen module `paged_attn` (export.cpp:1757-1764 equivalent), built with g++
    against torch's headers and linked to libpaged-attention.so (rpath $ORIGIN)."""
    import torch
    from torch.utils import cpp_extension as ce
    src = os.path.join(CSRC, "paged_attn_ext.cpp")
    out = ext_path()
    deps = [src, __file__, os.path.join(LIB, LIBNAME)] + _headers()
    if not force and _newer(out, deps):
        return out
    py_inc = sysconfig.get_paths()["include"]
    import pybind11
    incs = ce.include_paths() + [py_inc, pybind11.get_include(), "/opt/rocm/include", CSRC, INCLUDE]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-w",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=paged_attn",
           "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           *[f"-I{i}" for i in incs], src, "-o", out,
           f"-L{LIB}", "-l:" + LIBNAME, "-Wl,-rpath,$ORIGIN",
           *[f"-L{p}" for p in ce.library_paths()], "-lc10", "-ltorch", "-ltorch_cpu",
           "-ltorch_python", "-lc10_hip", "-ltorch_hip",
           "-L/opt/rocm/lib", "-lamdhip64"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"extension build failed:\n$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-ext", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    so = build_lib(a.jobs, a.force, a.verbose)
    print("built", so)
    if not a.no_variants:
        print("built", build_lib(a.jobs, a.force, a.verbose, variants=True))
    print("built", build_c_smoke(a.force))
    if not a.no_ext:
        print("built", build_ext(a.force, a.verbose))


if __name__ == "__main__":
    sys.exit(main())
