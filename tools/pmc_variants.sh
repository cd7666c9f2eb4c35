#!/bin/bash
# One PMC pass (instruction counts) per A/B variant of tools/_variants.json (run on the GPU box).
# usage: tools/pmc_variants.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
for name in $(python3 -c "import json; print(' '.join(json.load(open('tools/_variants.json'))))"); do
    lib=$(python3 -c "import json; print(json.load(open('tools/_variants.json'))['$name']['lib'])")
    ORBX_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d $OUT/$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing "$@" > $OUT/$name.log 2>&1
    python3 - "$OUT/$name" "$name" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
        d[(k, r["Counter_Name"])] += float(r["Counter_Value"])
ks = sorted({k for k, _ in d})
for k in ks:
    if k.startswith("k_"):
        print(sys.argv[2], k, " ".join(f"{c[8:]}={d[(k, c)]/1e6:.1f}M" for c in
              ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_WAVES"]))
PY
done
