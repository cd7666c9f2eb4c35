"""Per-kernel average of rocprofv3 --pmc counters (millions per dispatch, summed over the
dispatches of one step).  usage: python tools/pmc_summary.py CSV [CSV ...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("orbx::", "")
        c = r["Counter_Name"]
        agg[k][c] += float(r["Counter_Value"])
        disp[k][c].add((path, r["Dispatch_Id"]))
for k in sorted(agg):
    parts = []
    for c in sorted(agg[k]):
        n = len(disp[k][c])
        parts.append(f"{c}={agg[k][c] / 1e6:.1f}M/{n}")
    print(k, " ".join(parts))
