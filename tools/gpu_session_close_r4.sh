#!/bin/bash
# Closing check of the round: every GPU test, smoke(), the drop-in line and its kernel trace.
# usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --workload dropin --frames 300 > $OUT/dropin.json 2> $OUT/dropin.err || { echo "DROPIN BENCH FAILED"; tail -20 $OUT/dropin.err; exit 1; }
python - $OUT/dropin.json <<'PY'
import json, sys
j = json.load(open(sys.argv[1]))
for p in j["per_trackers"]: print("frame", p["trackers"], p["latency"]["median_ms"], round(p["pairs_per_s"]), p["sessions_agree"])
for p in j["two_thread_facade"]["per_trackers"]: print("facade", p["trackers"], p["latency"]["median_ms"], round(p["pairs_per_s"]))
print("digests_equal_one_call", j["two_thread_facade"]["digests_equal_one_call"])
PY
python tools/dropin_data.py /tmp/dd 8 > /dev/null && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_dropin -o run --output-format csv -- tests/native/facade_test bench /tmp/dd 100 20 1 frame > $OUT/prof_dropin.log 2>&1 || { echo "DROPIN TRACE FAILED"; exit 1; }
echo session done
