"""Fast A/B library variant: recompile only the named objects with extra flags, link them with
the default build's other objects, park the result as variants/lib_<name>.so (for
tools/lib_ab.py).  The default library is left untouched.

  python tools/quick_variant.py <name> "<flags>" [kind:hd:dt ...]     (default: bwd:128:bf16)
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from xf_flash_attention_cutlass_amd import build  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2].split()
    objs = sys.argv[3:] or ["bwd:128:bf16"]
    build.build_lib()                         # default objects up to date
    all_objs = sorted(os.path.join(build.OBJ, f) for f in os.listdir(build.OBJ) if f.endswith(".o"))
    tmp = tempfile.mkdtemp(prefix=f"xfa_{name}_")
    repl = {}
    for spec in objs:
        if ":" in spec:
            kind, hd, dt = spec.split(":")
            out = os.path.join(tmp, f"fmha_{kind}_hd{hd}_{dt}.o")
            defs = [f"-DXFA_HD={hd}", f"-DXFA_DTN={dt}", f"-DXFA_DT_BF16={1 if dt == 'bf16' else 0}"]
        else:                                 # a one-object kind (fwd_fp8)
            kind, defs = spec, []
            out = os.path.join(tmp, f"fmha_{kind}.o")
        src = os.path.join(build.CSRC, f"fmha_{kind}.hip")
        cmd = [build.HIPCC, *build.HIP_FLAGS, *flags, *defs, "-c", src, "-o", out]
        subprocess.run(cmd, check=True)
        repl[os.path.basename(out)] = out
    link = [repl.get(os.path.basename(o), o) for o in all_objs]
    os.makedirs(os.path.join(ROOT, "variants"), exist_ok=True)
    so = os.path.join(ROOT, "variants", f"lib_{name}.so")
    subprocess.run([build.HIPCC, f"--offload-arch={build.ARCH}", "-shared", "-fPIC", "-o", so, *link,
                    "-Wl,-soname,lib_" + name + ".so"], check=True)
    print(os.path.relpath(so, ROOT))


if __name__ == "__main__":
    main()
