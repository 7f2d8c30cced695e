"""CPU: the committed hand-scheduled asm bodies are exactly what their generators emit with the
default settings (tools/gen_fwd4.py -> fmha_fwd4_body.h, tools/gen_fwd8.py -> fmha_fwd8_body.h),
so a review of the generator is a review of the shipped kernel."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc")


@pytest.mark.parametrize("gen,body", [("gen_fwd4.py", "fmha_fwd4_body.h"),
                                      ("gen_fwd8.py", "fmha_fwd8_body.h")])
def test_generated_body_matches_generator(tmp_path, gen, body):
    out = tmp_path / body
    args = [sys.executable, os.path.join(ROOT, "tools", gen)]
    if gen == "gen_fwd4.py":
        args += ["--out", str(out)]
        subprocess.run(args, check=True, capture_output=True)
    else:
        code = (f"import sys; sys.path.insert(0, {os.path.join(ROOT, 'tools')!r}); "
                f"import gen_fwd8; gen_fwd8.emit({str(out)!r})")
        subprocess.run([sys.executable, "-c", code], check=True, capture_output=True)
    assert out.read_bytes() == open(os.path.join(CSRC, body), "rb").read()
