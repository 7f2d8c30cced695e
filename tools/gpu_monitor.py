"""Side-process GPU clock / power sampler for bench.py (record the clock the
box held over the timed region, so a slow lease can be told from a slow schedule).

Started by bench.py as a CHILD process before bench.py touches the GPU; this process never
initialises the GPU itself (it only runs `amd-smi metric`, a driver query, as its own children).
It appends one JSON line per sample to OUT:

    {"t": unix time, "gfx_mhz": [per-XCD current gfx clock], "power_w": socket power}

and stops when its stdin closes (the parent exited or closed the pipe) or after --max-s.
amd-smi numbers every GPU of the machine and ignores HIP_/ROCR_VISIBLE_DEVICES, so the parent,
once it knows its device's PCI address, writes a line `bdf DDDD:BB:DD` to this process' stdin:
sampling then moves to the amd-smi GPU with that BDF (from `amd-smi list`), and every sample
records the BDF it was taken from ("bdf": null until the parent's device is matched).

  python tools/gpu_monitor.py OUT.jsonl [--interval 0.1] [--gpu 0]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import threading
import time


def sample(amdsmi: str, gpu: int):
    r = subprocess.run([amdsmi, "metric", "-g", str(gpu), "-c", "-p", "--json"],
                       capture_output=True, text=True, timeout=10)
    d = json.loads(r.stdout)
    g = d["gpu_data"][0] if isinstance(d, dict) else d[0]
    clk = []
    for name, c in sorted(g.get("clock", {}).items()):
        if name.startswith("gfx_") and isinstance(c, dict):
            v = c.get("clk", {})
            if isinstance(v, dict) and isinstance(v.get("value"), (int, float)):
                clk.append(v["value"])
    pw = g.get("power", {}).get("socket_power", {})
    return clk, (pw.get("value") if isinstance(pw, dict) else None)


def bdf_index(amdsmi: str, bdf: str):
    """amd-smi's index of the GPU at PCI address `bdf` (DDDD:BB:DD, function optional)."""
    r = subprocess.run([amdsmi, "list", "--json"], capture_output=True, text=True, timeout=20)
    d = json.loads(r.stdout)
    items = d if isinstance(d, list) else next((v for v in d.values() if isinstance(v, list)), [])
    want = bdf.lower()
    for it in items:
        b = str(it.get("bdf", "")).lower()
        if b and b.startswith(want):
            return int(it["gpu"]), b
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--interval", type=float, default=0.1)
    ap.add_argument("--gpu", type=int, default=0)
    ap.add_argument("--max-s", type=float, default=900.0)
    a = ap.parse_args()
    amdsmi = shutil.which("amd-smi") or "/opt/rocm/bin/amd-smi"
    stop = threading.Event()
    target = {"gpu": a.gpu, "bdf": None}

    def watch_stdin():
        try:
            for line in sys.stdin:
                if line.startswith("bdf "):
                    try:
                        idx, b = bdf_index(amdsmi, line.split()[1])
                    except (OSError, ValueError, KeyError, TypeError, subprocess.SubprocessError):
                        idx, b = None, None
                    if idx is not None:
                        target.update(gpu=idx, bdf=b)
        except (OSError, ValueError):
            pass
        stop.set()

    threading.Thread(target=watch_stdin, daemon=True).start()
    t_end = time.time() + a.max_s
    fails = 0
    with open(a.out, "a") as f:
        while not stop.is_set() and time.time() < t_end and fails < 5:
            t = time.time()
            try:
                gpu, bdf = target["gpu"], target["bdf"]
                clk, pw = sample(amdsmi, gpu)
                fails = 0
                f.write(json.dumps({"t": round(t, 4), "gfx_mhz": clk, "power_w": pw, "gpu": gpu,
                                    "bdf": bdf}) + "\n")
                f.flush()
            except (OSError, ValueError, KeyError, IndexError, TypeError,
                    subprocess.SubprocessError):
                fails += 1
            stop.wait(max(0.0, a.interval - (time.time() - t)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
