"""Summarise rocprofv3 --pmc CSVs: per kernel name, mean over dispatches of each counter."""
import csv, glob, sys, collections
def load(d):
    rows = list(csv.DictReader(open(glob.glob(d + "/*counter_collection.csv")[0])))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
if __name__ == "__main__":
    want = sys.argv[2] if len(sys.argv) > 2 else "fmha"
    for d in sorted(glob.glob(sys.argv[1])):
        if not glob.glob(d + "/*counter_collection.csv"):
            continue
        for k, cs in load(d).items():
            if want in k:
                print(d.split("/")[-1], k[:60], {c: f"{v:.4g}" for c, v in sorted(cs.items())})
