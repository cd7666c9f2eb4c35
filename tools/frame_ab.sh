#!/bin/bash
# One-call stereo Frame A/B: zero-copy level 0 vs the H2D DMA (tuning lib, digests compared),
# and k_stereo's phase costs at one pair (ST_DIAG builds, kernel trace).  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd 8 > /dev/null || exit 1
B=$PWD/tests/native/facade_test
for zc in 0 1; do
  for K in 1 8; do
    F=$([ $K = 1 ] && echo 200 || echo 100)
    LD_LIBRARY_PATH=$PWD/tools/_var/tune:$LD_LIBRARY_PATH ORBX_FRAME_ZEROCOPY=$zc timeout -k 10 120 $B bench /tmp/dd $F 20 $K frame > $OUT/zc${zc}_k$K.json || exit 1
  done
done
python - $OUT <<'PY'
import json, sys
for n in ("zc0_k1", "zc1_k1", "zc0_k8", "zc1_k8"):
    j = json.load(open(f"{sys.argv[1]}/{n}.json")); v = sorted(j["latency_ms"])
    print(n, "median", v[len(v)//2], "pairs/s", round(j["trackers"]*j["frames"]/(j["wall_ms"]/1e3)), "digest", j["digests"][0], "agree", len(set(j["digests"])) == 1)
PY
for v in tune std3 std2 std1; do
  LD_LIBRARY_PATH=$PWD/tools/_var/$v:$LD_LIBRARY_PATH timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/st_$v -o run -- $B bench /tmp/dd 40 10 1 frame > $OUT/st_$v.log 2>&1 || { echo "TRACE $v FAILED"; tail -3 $OUT/st_$v.log; exit 1; }
  python - $OUT/st_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_stereo' in r['Name'] or 'octree' in r['Name']: print(sys.argv[2], r['Name'][:24], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
PY
done
