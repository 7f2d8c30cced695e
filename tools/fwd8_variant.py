"""A/B library variant of the 4-wave fp8 forward: compile fmha_fwd_fp8.hip against another
generated body and link it with the default build's other objects as variants/lib_<name>.so
(own soname; compare with tools/lib_ab.py --mode fwd_fp8).

  python tools/fwd8_variant.py <name> <body.h>
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from xf_flash_attention_cutlass_amd import build  # noqa: E402


def main():
    name, body = sys.argv[1], os.path.abspath(sys.argv[2])
    build.build_lib()
    obj = os.path.join(tempfile.mkdtemp(prefix=f"xfa8_{name}_"), "fmha_fwd_fp8.o")
    subprocess.run([build.HIPCC, *build.HIP_FLAGS, f'-DXFA_FWD8_BODY="{body}"', "-c",
                    os.path.join(build.CSRC, "fmha_fwd_fp8.hip"), "-o", obj], check=True)
    objs = [obj if f == "fmha_fwd_fp8.o" else os.path.join(build.OBJ, f)
            for f in sorted(os.listdir(build.OBJ)) if f.endswith(".o")]
    os.makedirs(os.path.join(ROOT, "variants"), exist_ok=True)
    so = os.path.join(ROOT, "variants", f"lib_{name}.so")
    subprocess.run([build.HIPCC, f"--offload-arch={build.ARCH}", "-shared", "-fPIC", "-o", so, *objs,
                    f"-Wl,-soname,lib_{name}.so"], check=True)
    print(os.path.relpath(so, ROOT))


if __name__ == "__main__":
    main()
