"""Summarize rocprofv3 kernel traces / PMC counters per kernel (and per k_level level)."""
import csv, sys, collections, os

def short(name):
    n = name.split("(")[0].replace("orbx::", "")
    return n

def trace(path):
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(list)
    for r in rows:
        n = short(r["Kernel_Name"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        key = n
        if n.startswith(("k_level", "void k_level")):
            key = f"k_level[grid={r.get('Grid_Size_X', r.get('Grid_Size', '?'))}]"
        per[key].append(d)
    print("== kernel trace (us per dispatch, mean) ==")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:40s} n={len(v):4d} mean={sum(v)/len(v)/1000:9.1f} total={sum(v)/1000:9.1f}")

def pmc(path):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        n = short(r["Kernel_Name"])
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n].add(r["Dispatch_Id"])
    for n, c in agg.items():
        nd = len(disp[n])
        print(n, nd, {k: f"{v/nd:.4g}" for k, v in sorted(c.items())})

if __name__ == "__main__":
    d = sys.argv[1]
    trace(os.path.join(d, "trace/run_kernel_trace.csv"))
    for p in ("pmc1", "pmc2", "pmc3", "pmc4"):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if os.path.exists(f):
            print(f"== {p} (per dispatch) ==")
            pmc(f)
