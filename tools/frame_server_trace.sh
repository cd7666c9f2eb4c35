#!/bin/bash
# The frame server at K = 4 / 8: batch sizes and device time (tuning lib, ORBX_FS_STATS), then a
# kernel + copy trace of the K = 8 loop: how busy the device is between batches.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd 32 > /dev/null || exit 1
B=$PWD/tests/native/facade_test
T=$PWD/tools/_var/tune
for stg in 1 2; do
  for K in 4 8; do
    LD_LIBRARY_PATH=$T:$LD_LIBRARY_PATH ORBX_FS_STATS=1 ORBX_STAGE_THREAD=$stg timeout -k 10 120 $B bench /tmp/dd 200 20 $K frame > $OUT/s${stg}_k$K.json 2> $OUT/s${stg}_k$K.err || { echo "RUN FAILED"; tail -3 $OUT/s${stg}_k$K.err; exit 1; }
    python - $OUT/s${stg}_k$K.json stage$stg K=$K <<'PY'
import json, sys
j = json.load(open(sys.argv[1])); v = sorted(j["latency_ms"])
print(sys.argv[2], sys.argv[3], "median", v[len(v)//2], "pairs/s", round(j["trackers"]*j["frames"]/(j["wall_ms"]/1e3)))
PY
    cat $OUT/s${stg}_k$K.err
  done
done
LD_LIBRARY_PATH=$T:$LD_LIBRARY_PATH ORBX_STAGE_THREAD=2 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr8 -o run -- $B bench /tmp/dd 100 20 8 frame > $OUT/tr8.log 2>&1 || { echo "TRACE FAILED"; tail -5 $OUT/tr8.log; exit 1; }
python - $OUT/tr8 <<'PY'
import csv, sys, collections
d = sys.argv[1]
ker = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")) for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv"))]
cp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"] if "Direction" in r else r.get("Operation", "copy")) for r in csv.DictReader(open(f"{d}/run_memory_copy_trace.csv"))]
allv = sorted(ker + cp)
a = allv[len(allv) // 5][0]; b = allv[4 * len(allv) // 5][0]
def union(iv):
    tot = 0; cur_s = cur_e = None
    for s, e, _ in sorted(iv):
        if s >= b or e <= a: continue
        s, e = max(s, a), min(e, b)
        if cur_e is None or s > cur_e:
            if cur_e is not None: tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else: cur_e = max(cur_e, e)
    if cur_e is not None: tot += cur_e - cur_s
    return tot
W = b - a
print(f"window {W/1e3:.0f} us: kernels busy {union(ker)/W:.2f}, copies busy {union(cp)/W:.2f}, either {union(ker+cp)/W:.2f}")
st = collections.defaultdict(lambda: [0, 0])
for s, e, n in ker + cp:
    if a <= s < b: st[n][0] += 1; st[n][1] += e - s
for n, (c, t) in sorted(st.items(), key=lambda x: -x[1][1]):
    print(f"  {n[:40]:40s} {c:6d} calls {t/c/1e3:8.1f} us mean {t/W:6.2f} of window")
PY
