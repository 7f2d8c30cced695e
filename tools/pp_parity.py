"""Run the forward GPU parity tests with a given fmha option set (e.g. fwd_pp=1)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytest
from xf_flash_attention_cutlass_amd import capi
for spec in sys.argv[1].split(","):
    n, v = spec.split("=")
    assert capi.lib().fmha_set_option(n.encode(), int(v)) == 0
sys.exit(pytest.main(["-q", "-m", "gpu", "-x", "tests/test_fwd_gpu.py"] + sys.argv[2:]))
