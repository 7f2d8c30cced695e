"""CPU: the committed hand-scheduled asm bodies are exactly what their generators emit with the
default settings (tools/gen_fwd4.py -> fmha_fwd4_body.h, tools/gen_fwd8.py -> fmha_fwd8_body.h,
tools/gen_fwdpp.py -> fmha_fwdpp_body.h, tools/gen_fwdpp16.py -> fmha_fwdpp16_body.h,
tools/gen_fwd8pp.py -> fmha_fwd8pp_body.h),
so a review of the generator is a review of the shipped kernel."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "xf_flash_attention_cutlass_amd", "csrc")


@pytest.mark.parametrize("gen,body", [("gen_fwd4.py", "fmha_fwd4_body.h"),
                                      ("gen_fwd8.py", "fmha_fwd8_body.h"),
                                      ("gen_fwdpp.py", "fmha_fwdpp_body.h"),
                                      ("gen_fwdpp16.py", "fmha_fwdpp16_body.h"),
                                      ("gen_fwd8pp.py", "fmha_fwd8pp_body.h")])
def test_generated_body_matches_generator(tmp_path, gen, body):
    out = tmp_path / body
    args = [sys.executable, os.path.join(ROOT, "tools", gen)]
    if gen in ("gen_fwd4.py", "gen_fwdpp.py", "gen_fwdpp16.py", "gen_fwd8pp.py"):
        args += ["--out", str(out)]
        subprocess.run(args, check=True, capture_output=True)
    else:
        code = (f"import sys; sys.path.insert(0, {os.path.join(ROOT, 'tools')!r}); "
                f"import gen_fwd8; gen_fwd8.emit({str(out)!r})")
        subprocess.run([sys.executable, "-c", code], check=True, capture_output=True)
    assert out.read_bytes() == open(os.path.join(CSRC, body), "rb").read()


@pytest.mark.parametrize("body", ["fmha_fwd4_body.h", "fmha_fwd8_body.h", "fmha_fwdpp_body.h",
                                  "fmha_fwdpp16_body.h", "fmha_fwd8pp_body.h"])
def test_return_addresses_guarded(body):
    """Every s_getpc_b64 return address in the generated bodies has an assembler guard that pins
    the sign of its offset (the redo fault of round 4 came from a stub moved
    before/after its return point with the high word's sign assumed)."""
    lines = [ln.strip().strip('"').replace("\\n", "") for ln in
             open(os.path.join(CSRC, body)).read().splitlines()]
    guards = {ln for ln in lines if ln.startswith(".if (")}
    pcs = [i for i, ln in enumerate(lines) if ln.startswith("s_getpc_b64")]
    assert pcs
    for i in pcs:
        lab = lines[i + 1].rstrip(":")                    # .Lpc.../.Lpe... label after s_getpc
        add = lines[i + 2]                                # s_add_u32 sX, sX, .Lret - .Lpc
        ret = add.split(", ")[-1].split(" - ")[0]
        hi = lines[i + 3]
        cond = ">= 0" if hi.endswith("-1") else "< 0"
        assert hi.startswith("s_addc_u32") and hi.endswith(("-1", " 0")), lines[i:i + 4]
        assert f".if ({ret} - {lab}) {cond}" in guards, (ret, lab, cond)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
@pytest.mark.parametrize("back,ret_first,ok", [(True, True, True), (False, False, True),
                                               (False, True, False), (True, False, False)])
def test_return_address_guard_assembles(tmp_path, back, ret_first, ok):
    """The guard really fires: a stub whose return point lies on the other side than the sign it
    assumes fails to assemble (the guards sit at the end of the statement, as the generators
    emit them)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_fwd4
    gen_fwd4.GUARDS.clear()
    stub = ["s_getpc_b64 s[10:11]", ".Lpc%=:", "s_add_u32 s10, s10, .Lret%= - .Lpc%="]
    stub += gen_fwd4.addc_ret(11, ".Lret%=", ".Lpc%=", back) + ["s_setpc_b64 s[10:11]"]
    ret = [".Lret%=:", "v_mov_b32 v1, 0", "s_branch .Lend%="]
    body = (["s_branch .Lx%="] + ret + [".Lx%=:"] + stub if ret_first else
            ["s_branch .Lx%="] + [".Lx%=:"] + stub + ret)
    body += [".Lend%=:"] + gen_fwd4.GUARDS
    gen_fwd4.GUARDS.clear()
    src = tmp_path / "t.hip"
    src.write_text("#include <hip/hip_runtime.h>\n__global__ void k(int* o) {\n  asm volatile(\n" +
                   "".join(f'    "{b}\\n"\n' for b in body) +
                   '    ::: "s10", "s11", "v1");\n}\n')
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-c",
                        str(src), "-o", str(tmp_path / "t.o")], capture_output=True, text=True)
    assert (r.returncode == 0) == ok, r.stderr[-500:]
    if not ok:
        assert ".err" in r.stderr
