import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session", autouse=True)
def _tuning_options():
    """XFA_TEST_OPTIONS="name=value,..." runs the suite under fmha_set_option knobs (A/B builds
    and schedules get the same parity coverage as the defaults)."""
    spec = os.environ.get("XFA_TEST_OPTIONS", "")
    if spec:
        from xf_flash_attention_cutlass_amd import capi
        for o in spec.split(","):
            name, val = o.split("=")
            assert capi.lib().fmha_set_option(name.encode(), int(val)) == 0, name
    yield


_REPORT = []


@pytest.fixture(scope="session")
def parity_report():
    """Collects {case, metric, err, bound} rows; XFA_PARITY_REPORT=<path> writes them as JSON
    at the end of the session (the committed profiles/r*_parity.json evidence)."""
    yield _REPORT.append
    path = os.environ.get("XFA_PARITY_REPORT")
    if path and _REPORT:
        import json
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(_REPORT, f, indent=1)
