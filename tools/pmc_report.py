"""Summarise tools/pmc_round.sh output into the committed roofline evidence:

  profiles/<tag>_pmc.json      per mode, per fmha kernel: mean counters over dispatches and the
                               derived figures (effective clock, MFMA utilisation from
                               SQ_INSTS_MFMA, VALU per MFMA, wait / LDS-conflict fractions,
                               HBM bytes per launch)
  profiles/<tag>_traffic.json  per mode: HBM bytes per launch of the dominant kernel (the
                               "traffic" field bench.py reads)
  profiles/<tag>_<mode>_kernel_stats.csv   the kernel-trace --stats summary of the same command

Derivations (MI355X_MICROARCH.md):
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel cycles = GRBM_GUI_ACTIVE / 8;
    effective clock = cycles / dispatch duration, reported only for dispatches of >= 50 us
    (GRBM_GUI_ACTIVE counts the dispatch's ramp and drain beside it: on ~5 us kernels the
    quotient read 5.5-5.7 GHz in r04); shorter kernels get null, and no utilisation derived
    from the clock;
  * v_mfma_f32_32x32x16 holds one SIMD's matrix pipe for 32 cycles, 16x16x32 for 16, the
    block-scaled fp8 v_mfma_scale_f32_32x32x64_f8f6f4 for 64 (twice the bf16 form's cycles at 4x
    the K; the fp8 kernels issue only that one): MFMA utilisation = SQ_INSTS_MFMA x 32 (64) / (4 SIMDs x
    CUs x cycles) - an upper bound for kernels that also issue 16x16x32 (the backward's dQ);
  * FETCH_SIZE reports half the bytes of wide streaming reads on gfx950: x2; WRITE_SIZE exact
    for 16-B/lane stores and float atomics; both in KiB;
  * SQ_WAIT_ANY / SQ_WAVE_CYCLES = fraction of wave time parked on s_waitcnt / barriers.

  python tools/pmc_report.py gpurun_out/prof r03 fwd fwdbwd varlen decode fwd_fp8
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

NUM_CUS = 256
MIN_CLOCK_NS = 50_000      # shortest dispatch whose GRBM cycles / duration is read as a clock


def counters(d):
    """{kernel: {counter: mean}, '__dur__': mean ns} over the dispatches of every fmha kernel."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "fmha" not in k:
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs[k][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {}
    for k, cs in vals.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        ds = list(durs[k].values())
        out[k]["__dur_ns__"] = sum(ds) / len(ds)
        out[k]["__dispatches__"] = len(ds)
    return out


def stats(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    return (list(csv.DictReader(open(f[0]))), f[0]) if f else ([], None)


def trace_median_ns(d, kernel):
    """Median dispatch duration (ns) of `kernel` from the kernel-trace csv of the stats run."""
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        return None
    ds = sorted(float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                for r in csv.DictReader(open(f[0])) if r["Kernel_Name"] == kernel)
    return ds[len(ds) // 2] if ds else None


def stats_run_line(root, m):
    """The bench JSON line the profiled stats run itself printed (same process as the kernel
    trace: its ms_per_step is the step the trace's kernel median belongs to)."""
    f = os.path.join(root, f"{m}_stats.out")
    if not os.path.exists(f):
        return None
    lines = [x for x in open(f) if x.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def short(name):
    return name.split("(")[0].replace("void ", "")[:120]


def main():
    root, tag, modes = sys.argv[1], sys.argv[2], sys.argv[3:]
    pmc, traffic = {}, {}
    for m in modes:
        rows, sf = stats(os.path.join(root, f"{m}_stats"))
        if sf:
            shutil.copy(sf, os.path.join("profiles", f"{tag}_{m}_kernel_stats.csv"))
        dom = max(rows, key=lambda r: float(r["TotalDurationNs"])) if rows else None
        med = trace_median_ns(os.path.join(root, f"{m}_stats"), dom["Name"]) if dom else None
        merged = collections.defaultdict(dict)
        for p in ("sq1", "sq2", "fetch", "write"):
            for k, cs in counters(os.path.join(root, f"{m}_{p}")).items():
                for c, v in cs.items():
                    if c.startswith("__"):
                        merged[k].setdefault(c + p, v)
                    else:
                        merged[k][c] = v
        res = {}
        for k, c in merged.items():
            e = {"dispatches_profiled": int(c.get("__dispatches__sq1", 0))}
            cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
            dur = c.get("__dur_ns__sq1", 0)
            long_enough = bool(cyc and dur >= MIN_CLOCK_NS)
            if cyc and dur:
                e["kernel_cycles"] = round(cyc)
                e["profiled_duration_us"] = round(dur / 1e3, 2)
                e["effective_clock_ghz"] = round(cyc / dur, 3) if long_enough else None
            if long_enough and "SQ_INSTS_MFMA" in c:
                # cycles per MFMA instruction: 64 for the block-scaled fp8 one, 16 for
                # v_mfma_f32_16x16x32 (the M16 ping-pong body, the 16-row decode tile), else 32
                m16 = re.search(r"fmha_fwdpp_kernel<(true|false), true", k) is not None
                per = 64 if "fp8" in k or "fwd8" in k else 16 if (m16 or "decode" in k) else 32
                e["mfma_util_from_insts"] = round(c["SQ_INSTS_MFMA"] * per / (4 * NUM_CUS * cyc), 4)
            if c.get("SQ_INSTS_MFMA"):
                e["valu_per_mfma"] = round(c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"], 2)
                e["lds_insts_per_mfma"] = round(c.get("SQ_INSTS_LDS", 0) / c["SQ_INSTS_MFMA"], 2)
            if c.get("SQ_WAVE_CYCLES"):
                e["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 4)
            if c.get("SQ_ACTIVE_INST_ANY") and c.get("SQ_WAIT_INST_ANY"):
                e["wait_inst_over_active"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_ACTIVE_INST_ANY"], 4)
            if c.get("SQ_LDS_IDX_ACTIVE"):
                e["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) /
                                                    c["SQ_LDS_IDX_ACTIVE"], 4)
            if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
                rd = 2 * c.get("FETCH_SIZE", 0) * 1024
                wr = c.get("WRITE_SIZE", 0) * 1024
                e["hbm_read_bytes_x2corr"] = int(rd)
                e["hbm_write_bytes"] = int(wr)
                e["hbm_bytes_per_launch"] = int(rd + wr)
            e["counters_mean"] = {x: round(v, 1) for x, v in sorted(c.items()) if not x.startswith("__")}
            res[short(k)] = e
        line = stats_run_line(root, m)
        pmc[m] = {"dominant_kernel": short(dom["Name"]) if dom else None,
                  "stats_run_ms_per_step": line["ms_per_step"] if line else None,
                  "dominant_avg_ns": float(dom["AverageNs"]) if dom else None,
                  "dominant_median_ns": med,
                  "dominant_calls": int(dom["Calls"]) if dom else None,
                  "kernels": res}
        if dom:
            key = next((k for k in res if k == short(dom["Name"])), None)
            if key and "hbm_bytes_per_launch" in res[key]:
                traffic[m] = {"kernel": key, "avg_ns": float(dom["AverageNs"]), "median_ns": med,
                              "stats_run_ms_per_step": line["ms_per_step"] if line else None,
                              "calls": int(dom["Calls"]),
                              "hbm_bytes_per_launch": res[key]["hbm_bytes_per_launch"],
                              "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + "
                                      "WRITE_SIZE, KiB->B; Infinity-Cache hits are counted"}
    json.dump(pmc, open(os.path.join("profiles", f"{tag}_pmc.json"), "w"), indent=1)
    json.dump(traffic, open(os.path.join("profiles", f"{tag}_traffic.json"), "w"), indent=1)
    for m, d in pmc.items():
        print(m, d["dominant_kernel"], d["dominant_avg_ns"])
        for k, e in d["kernels"].items():
            print("  ", k[:70], {x: y for x, y in e.items() if x != "counters_mean"})


if __name__ == "__main__":
    main()
