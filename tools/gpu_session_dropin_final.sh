#!/bin/bash
# Drop-in line of record: parity of the facade / one-call frame, bench.py --workload dropin, and
# the frame-path A/B on hot (8 pairs) and cold (32 pairs) images.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_facade_cpp.py tests/test_gpu_extract.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --workload dropin > $OUT/dropin.json 2> $OUT/dropin.err || { echo "DROPIN BENCH FAILED"; tail -20 $OUT/dropin.err; exit 1; }
cat $OUT/dropin.json
python tools/dropin_data.py /tmp/dd 8 > /dev/null || exit 1
python tools/dropin_data.py /tmp/dd32 32 > /dev/null || exit 1
export ORBX_AB_SETTINGS=${AB:-default,frame,frame_nostage,frame_stage2,frame_solo}
echo "== hot (8 pairs)"
timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd 1,2,8 > $OUT/ab_hot.txt 2>&1 || { echo "AB FAILED"; tail -5 $OUT/ab_hot.txt; exit 1; }
cat $OUT/ab_hot.txt
echo "== cold (32 pairs)"
timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd32 1,8 > $OUT/ab_cold.txt 2>&1 || { echo "AB FAILED"; tail -5 $OUT/ab_cold.txt; exit 1; }
cat $OUT/ab_cold.txt
