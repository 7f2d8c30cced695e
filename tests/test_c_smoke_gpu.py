"""GPU: the torch-free C++ caller (tests/c_smoke.cpp, built by build.py into tests/bin/c_smoke
and linked only against libpaged-attention.so) runs fmha_fwd, fmha_varlen_fwd,
fmha_page_kvcache_fwd and fmha_bwd on a committed golden case (the reference test.py's live
configuration B1 H1 S128 D128 fp16 causal, test.py:711-750) and checks each against the oracle
with the reference's pass rules (2x the low-precision error for O, test.py:975; 3x + 1e-5 for
the gradients, test.py:984-986).  This test only dumps the fixture as raw bytes, computes the
bounds with the oracle on the CPU and reads the program's verdict."""
import os
import subprocess

import pytest
import torch

from oracle import attention_ref as orc
from tests import golden_util as gu

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "bin", "c_smoke")


@pytest.mark.parametrize("name", ["fwd_f16_b1h1s128d128_causal", "fwd_bf16_b1h4hk2_q113k203_d128"])
def test_c_caller_golden(tmp_path, name):
    assert os.path.exists(BIN), "tests/bin/c_smoke missing: run xf_flash_attention_cutlass_amd/build.py"
    t, m = gu.load(name)
    assert not m["alibi"] and m["softcap"] == 0 and tuple(m["window"]) == (-1, -1)
    fp16 = t["q"].dtype == torch.float16
    for key in ("q", "k", "v", "dout"):
        t[key].contiguous().view(torch.int16).numpy().tofile(str(tmp_path / f"{key}.bin"))
    for key in ("out_ref", "dq_ref", "dk_ref", "dv_ref"):
        t[key].float().contiguous().numpy().tofile(str(tmp_path / f"{key}.bin"))
    fwd_bound = 2 * (t["out_pt"].float() - t["out_ref"].float()).abs().max().item()
    # gradient bounds: the low-precision twin of the oracle (the pinned restatement, as
    # tests/test_bwd_gpu.py does)
    qq, kk, vv = (t[x].clone().requires_grad_(True) for x in ("q", "k", "v"))
    out, _ = orc.attention_ref(qq, kk, vv, causal=m["causal"], upcast=False, reorder_ops=True)
    pt = torch.autograd.grad(out, (qq, kk, vv), t["dout"])
    gb = [3 * (p.float() - t[n + "_ref"].float()).abs().max().item() + 1e-5
          for n, p in zip(("dq", "dk", "dv"), pt)]
    scale = m["d"] ** -0.5
    (tmp_path / "meta.txt").write_text(
        f"{m['b']} {m['h']} {m['hk']} {m['sq']} {m['sk']} {m['d']} {int(m['causal'])} {int(fp16)} "
        f"{scale!r} {fwd_bound!r} {gb[0]!r} {gb[1]!r} {gb[2]!r}\n")
    r = subprocess.run([BIN, str(tmp_path)], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0 and "C_SMOKE_OK" in r.stdout, r.stdout + r.stderr
