"""Loading helpers for the committed golden fixtures (tests/golden/*.safetensors)."""
import glob
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names(kind=None):
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "*.safetensors"))):
        n = os.path.basename(f)[: -len(".safetensors")]
        if kind is None or meta(n)["kind"] == kind:
            out.append(n)
    return out


def meta(name):
    from safetensors import safe_open
    with safe_open(os.path.join(GOLDEN, name + ".safetensors"), "pt") as f:
        return json.loads(f.metadata()["meta"])


def load(name):
    from safetensors.torch import load_file
    return load_file(os.path.join(GOLDEN, name + ".safetensors")), meta(name)
