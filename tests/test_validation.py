"""CPU: host-side guards of the C ABI and the Python wrappers, reached with fake pointers (no
kernel is launched): the 32-bit slab limit (fmha_api.cpp slab_ok), the deterministic
backward's workspace size, and the fp8 wrapper refusing options it cannot honour."""
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


def _acc(tok, h):
    return -(-(tok * h * 128 * 4) // 256) * 256         # fp32 [tokens][h][128], 256-B rounded


def _dsum(tok, h):
    return -(-(tok * h * 4) // 256) * 256


def _cus(L):
    """The CU count the library sizes for (the live device's, 256 without one): the slice count
    of b * hk = 1 over a key range longer than CUs x 256 keys."""
    ws = L.fmha_bwd_workspace_size(256, 1 << 20, 1, 1, 1, 128, True)
    return (ws - _dsum(256, 1)) // _acc(256, 1)


def test_deterministic_bwd_workspace_bounded():
    """deterministic=True: S = min(ceil(CUs / (b * hk)), key blocks) dQ slices (export.cpp:1090-1091's
    bound; no workgroup walks more slices than there are 256-key blocks), capped at 8 GiB of
    slices beyond the first, so the workspace stops growing with seqlen_k.  Beside the
    slices: D = rowsum(dO O) and the causal-ALiBi LSE in the kernels' convention, fp32 per row."""
    L = capi.lib()
    cus = _cus(L)
    assert cus >= 1
    for b, h, hk, sq in ((4, 32, 32, 16384), (1, 16, 16, 45056), (8, 32, 8, 1024), (1, 1, 1, 4096),
                         (1, 64, 1, 2048), (2, 32, 4, 4096)):
        tok = b * sq
        for sk in (128, 4096, 65536, 1 << 20):
            nkb = -(-sk // 256)
            slices = min(-(-cus // (b * hk)), nkb, 1 + (8 << 30) // _acc(tok, h))
            want = slices * _acc(tok, h) + 2 * _dsum(tok, h)
            assert L.fmha_bwd_workspace_size(sq, sk, b, h, hk, 128, True) == want, (b, h, hk, sq, sk)
            assert L.fmha_varlen_bwd_workspace_size(tok, sk, b, h, hk, 128, True) == want
        assert L.fmha_bwd_workspace_size(sq, 4096, b, h, hk, 128, False) == _acc(tok, h) + 2 * _dsum(tok, h)
    # MQA, one sequence of 32k tokens x 64 query heads (1 GiB per slice): the byte cap bounds it
    # (the CU bound alone asked for 256 slices = 256 GiB)
    ws = L.fmha_bwd_workspace_size(32768, 32768, 1, 64, 1, 128, True)
    assert ws <= 9 * _acc(32768, 64) + 2 * _dsum(32768, 64)
    # B4 H32 S16384 D128: at most two slices on a 256-CU device
    assert L.fmha_bwd_workspace_size(16384, 16384, 4, 32, 32, 128, True) <= (
        max(2, -(-cus // 128)) * _acc(4 * 16384, 32) + 2 * _dsum(4 * 16384, 32))


@pytest.mark.parametrize("kw", [dict(dropout_p=0.1), dict(softcap=30.0),
                                dict(alibi_slopes=torch.zeros(2))])
def test_fp8_wrapper_refuses_unsupported_options(kw):
    from xf_flash_attention_cutlass_amd.interface import flash_attn_func
    q = torch.zeros(1, 16, 2, 128, dtype=torch.float8_e4m3fn)
    with pytest.raises(NotImplementedError):
        flash_attn_func(q, q, q, **kw)


def test_misaligned_pointers_and_strides_rejected():
    """The kernels move 16-byte chunks: the C ABI refuses bases that are not 16-byte aligned and
    (strided entry) strides that are not multiples of 8 elements, instead of faulting."""
    L = capi.lib()
    L.fmha_fwd(FAKE + 2, FAKE, FAKE, FAKE, None, 128, 128, 1, 4, 4, 128, 0.0, None, None,
               0.088, None, None, -1, -1, 0.0, False, False, 1)
    st, msg = _status()
    assert st != 0 and "16-byte aligned" in msg
    L.fmha_bwd(FAKE, FAKE, FAKE, FAKE + 8, FAKE, FAKE, FAKE, FAKE, FAKE, None, None, 128, 128, 1,
               4, 4, 128, 0.0, 0.088, -1, -1, 0.0, False, False, None, None, 0)
    st, msg = _status()
    assert st != 0 and "16-byte aligned" in msg
    import ctypes
    strides = (ctypes.c_int64 * 12)(128 * 4 * 128, 4 * 128 + 4, 128, 128 * 4 * 128, 4 * 128, 128,
                                    128 * 4 * 128, 4 * 128, 128, 128 * 4 * 128, 4 * 128, 128)
    L.fmha_fwd_strided(FAKE, FAKE, FAKE, FAKE, None, None, 128, 128, 2, 4, 4, 128, strides, 0.088,
                       -1, -1, 0.0, False, 1, None, 0.0, None)
    st, msg = _status()
    assert st != 0 and "multiples of 8 elements" in msg and "stride 1" in msg


def test_softcap_with_dropout_rejected():
    """The reference refuses softcap together with dropout (export.cpp:515,737,
    flash_api_hip.cpp:400,606,895,1128); so does every C entry that takes both."""
    L = capi.lib()
    L.fmha_fwd(FAKE, FAKE, FAKE, FAKE, None, 128, 128, 1, 4, 4, 128, 0.1, None, None, 0.088, None,
               None, -1, -1, 30.0, False, False, 1)
    st, msg = _status()
    assert st != 0 and "Softcapping does not support dropout" in msg
    L.fmha_bwd(FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, FAKE, None, None, 128, 128, 1, 4, 4,
               128, 0.1, 0.088, -1, -1, 30.0, False, False, None, None, 0)
    st, msg = _status()
    assert st != 0 and "Softcapping does not support dropout" in msg
