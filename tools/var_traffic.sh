#!/bin/bash
# Per-variant FETCH_SIZE / WRITE_SIZE passes (tools/variants.py libraries), one rocprofv3 run
# per counter and variant.  usage: tools/var_traffic.sh OUT NAME...
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
for v in "$@"; do
  export ORBX_LIB=my_orb_slam2_amd/liborbx_$v.so
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 --serial-steps 0 > $OUT/f_$v.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 --serial-steps 0 > $OUT/w_$v.log 2>&1
  python3 - $OUT $v <<'PY'
import csv, glob, sys, collections
out, v = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float); ids = collections.defaultdict(set)
for kind in ("f", "w"):
    for f in glob.glob(f"{out}/{kind}_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1]
            tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            ids[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k in sorted({k for k, _ in tot}):
    if not k.startswith("k_"):
        continue
    fs, ws = tot.get((k, "FETCH_SIZE"), 0.0), tot.get((k, "WRITE_SIZE"), 0.0)
    # two steps ran (warm-up + timed): per step = half; FETCH_SIZE x2 (gfx950), KiB -> GB
    print(f"{v:14s} {k:22s} traffic/step {(2 * fs + ws) * 1024 / 2 / 1e9:.3f} GB")
PY
done
