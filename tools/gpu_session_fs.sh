#!/bin/bash
# Frame-server iteration: its parity tests, then tools/frame_server_trace.sh and the frame A/B
# (cold pairs).  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_facade_cpp.py tests/test_gpu_extract.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/frame_server_trace.sh $1/tr || exit 1
python tools/dropin_data.py /tmp/dd32 32 > /dev/null || exit 1
ORBX_AB_SETTINGS=${AB:-frame,frame_nostage,frame_stage2} timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd32 1,2,4,8 > $OUT/ab_cold.txt 2>&1 || { echo "AB FAILED"; tail -5 $OUT/ab_cold.txt; exit 1; }
cat $OUT/ab_cold.txt
