#!/bin/bash
# The drop-in line of record (bench.py --workload dropin) and K = 8 repeats of the frame path
# (300 frames per session, cold pairs), interleaved with the stage-thread variants.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload dropin > $OUT/dropin.json 2> $OUT/dropin.err || { echo "DROPIN BENCH FAILED"; tail -20 $OUT/dropin.err; exit 1; }
python - $OUT/dropin.json <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
for p in j["per_trackers"]: print("frame", p["trackers"], p["latency"]["median_ms"], round(p["pairs_per_s"]), p["sessions_agree"])
for p in j["two_thread_facade"]["per_trackers"]: print("facade", p["trackers"], p["latency"]["median_ms"], round(p["pairs_per_s"]), p["sessions_agree"])
print("digests_equal_one_call", j["two_thread_facade"]["digests_equal_one_call"])
PY
python tools/dropin_data.py /tmp/dd32 32 > /dev/null || exit 1
B=$PWD/tests/native/facade_test
for rep in 1 2 3; do
  for stg in 1 0 2; do
    LD_LIBRARY_PATH=$PWD/tools/_var/tune:$LD_LIBRARY_PATH ORBX_STAGE_THREAD=$stg timeout -k 10 120 $B bench /tmp/dd32 300 30 8 frame > $OUT/r${rep}_s$stg.json || { echo "RUN FAILED"; exit 1; }
    python - $OUT/r${rep}_s$stg.json rep$rep stage$stg <<'PY'
import json, sys
j = json.load(open(sys.argv[1])); v = sorted(j["latency_ms"])
print(sys.argv[2], sys.argv[3], "K=8 median", v[len(v)//2], "mean", round(sum(v)/len(v), 4), "pairs/s", round(j["trackers"]*j["frames"]/(j["wall_ms"]/1e3)))
PY
  done
done
