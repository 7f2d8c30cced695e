"""Turn the PMC passes of tools/profile_round.sh into per-launch HBM bytes of each mode's
dominant kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of wide
streaming reads on gfx950 -> x2; WRITE_SIZE exact for 16 B/lane stores).  FETCH_SIZE and
WRITE_SIZE are in KiB (rocprofv3 derived counters).

  python tools/traffic.py gpurun_out/prof r01 fwd decode ...   -> profiles/r01_traffic.json
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def dominant(d):
    """Kernel with the largest total duration in the kernel-trace stats CSV."""
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    return r["Name"], float(r["AverageNs"]), int(r["Calls"])


def main():
    root, tag, modes = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = {}
    for m in modes:
        name, avg_ns, calls = dominant(os.path.join(root, f"{m}_stats"))
        fetch = per_kernel(os.path.join(root, f"{m}_fetch"), "FETCH_SIZE")
        write = per_kernel(os.path.join(root, f"{m}_write"), "WRITE_SIZE")
        key = next((k for k in fetch if k.split("(")[0] == name.split("(")[0]), None)
        if key is None and fetch:     # stats and counter CSVs may differ in demangling
            key = max(fetch, key=fetch.get)
        if key is None:
            continue
        rd = 2 * fetch[key] * 1024
        wr = write.get(key, 0.0) * 1024
        out[m] = {"kernel": name[:160], "avg_ns": avg_ns, "calls": calls,
                  "fetch_bytes_corrected": rd, "write_bytes": wr,
                  "hbm_bytes_per_launch": int(rd + wr),
                  "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->B; "
                          "Infinity-Cache hits are counted by these counters"}
    path = os.path.join("profiles", f"{tag}_traffic.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
