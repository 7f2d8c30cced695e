"""CPU: host-side guards of the C ABI and the Python wrappers, reached with fake pointers (no
kernel is launched): the 32-bit slab limit (fmha_api.cpp slab_ok), the deterministic
backward's workspace bound, and the fp8 wrapper refusing options it cannot honour."""
import pytest
import torch

from xf_flash_attention_cutlass_amd import capi

FAKE = 0x1000          # never dereferenced: every case fails validation before a launch


def _status():
    L = capi.lib()
    return L.fmha_last_status(), L.fmha_last_error().decode()


def test_fwd_slab_guard():
    # one sequence of 2^24 tokens x 64 heads x d128 bf16 = 256 GiB > the 2 GiB slab limit
    L = capi.lib()
    L.fmha_fwd(FAKE, FAKE, FAKE, FAKE, None, 1 << 24, 128, 1, 64, 64, 128, 0.0, None, None,
               0.088, None, None, -1, -1, 0.0, False, False, 1)
    st, msg = _status()
    assert st != 0 and "32-bit offsets" in msg and "q/o" in msg


def test_fwd_slab_guard_kv_side():
    L = capi.lib()
    L.fmha_fwd(FAKE, FAKE, FAKE, FAKE, None, 128, 1 << 24, 1, 64, 64, 128, 0.0, None, None,
               0.088, None, None, -1, -1, 0.0, False, False, 1)
    st, msg = _status()
    assert st != 0 and "k/v" in msg


def test_varlen_fwd_slab_guard():
    L = capi.lib()
    L.fmha_varlen_fwd(FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, 1 << 24, 128, 1, 64, 64, 128, None,
                      0.088, False, False, -1, -1)
    st, msg = _status()
    assert st != 0 and "32-bit offsets" in msg


def test_bwd_slab_guard_dq_accum():
    # q/o fit (h=1: 2^22 x 128 x 2 B = 1 GiB), the fp32 accumulator (2 GiB) does not
    L = capi.lib()
    sq = 1 << 22
    L.fmha_bwd(FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, None, None, sq, 128, 1, 1, 1,
               128, 0.0, 0.088, -1, -1, 0.0, False, False, None, None, 0)
    st, msg = _status()
    assert st != 0 and "dq_accum" in msg


def test_varlen_bwd_slab_guard_dq_accum():
    L = capi.lib()
    sq = 1 << 22
    L.fmha_varlen_bwd(FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, None, 0,
                      sq, 128, sq, 128, 1, 1, 1, 128, 0.088, -1, -1, 0.0, False, False, None,
                      None, 0, None, 0.0)
    st, msg = _status()
    assert st != 0 and "dq_accum" in msg


def test_deterministic_bwd_workspace_bound():
    # b8 h32 s32768 d128: one 1 GiB-per-slice x 128 key blocks -> far above the 32 GiB limit
    L = capi.lib()
    L.fmha_bwd(FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, None, None, 32768, 32768, 8,
               32, 32, 128, 0.0, 0.088, -1, -1, 0.0, True, False, None, None, 0)
    st, msg = _status()
    assert st != 0 and "deterministic" in msg
    # the same shape without determinism passes validation (the launch itself is not reached:
    # check only that the bound is what refused it, via the workspace-size query)
    need = L.fmha_bwd_workspace_size(32768, 32768, 8, 32, 32, 128, True)
    assert need > (32 << 30)
    assert L.fmha_bwd_workspace_size(32768, 32768, 8, 32, 32, 128, False) < need


@pytest.mark.parametrize("kw", [dict(dropout_p=0.1), dict(softcap=30.0),
                                dict(alibi_slopes=torch.zeros(2))])
def test_fp8_wrapper_refuses_unsupported_options(kw):
    from xf_flash_attention_cutlass_amd.interface import flash_attn_func
    q = torch.zeros(1, 16, 2, 128, dtype=torch.float8_e4m3fn)
    with pytest.raises(NotImplementedError):
        flash_attn_func(q, q, q, **kw)
