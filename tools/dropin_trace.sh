#!/bin/bash
# Drop-in host path: where a stereo frame's time goes (kernel + HIP API + copy traces at K=1 and
# K=8).  usage: tools/dropin_trace.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd 8 > /dev/null || exit 1
B=tests/native/boundary_test
timeout -k 10 120 $B bench /tmp/dd 300 30 1 > $OUT/k1.json || exit 1
timeout -k 10 120 $B bench /tmp/dd 100 20 8 > $OUT/k8.json || exit 1
python - $OUT <<'PY'
import json, sys
for n in ("k1", "k8"):
    j = json.load(open(f"{sys.argv[1]}/{n}.json")); v = sorted(j["latency_ms"])
    print(n, "median", v[len(v)//2], "mean", sum(v)/len(v), "pairs/s", j["trackers"]*j["frames"]/(j["wall_ms"]/1e3))
PY
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr1 -o run -- $B bench /tmp/dd 60 10 1 > $OUT/tr1.log 2>&1 || { echo "TRACE K=1 FAILED"; tail -5 $OUT/tr1.log; exit 1; }
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr8 -o run -- $B bench /tmp/dd 30 10 8 > $OUT/tr8.log 2>&1 || { echo "TRACE K=8 FAILED"; tail -5 $OUT/tr8.log; exit 1; }
echo done
