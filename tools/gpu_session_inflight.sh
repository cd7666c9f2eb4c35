#!/bin/bash
# Frame server with two batches in flight: parity tests, then interleaved A/B against one batch
# at a time (ORBX_FS_INFLIGHT=1), 32 cold pairs.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_facade_cpp.py tests/test_gpu_extract.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
python tools/dropin_data.py /tmp/dd32 32 > /dev/null || exit 1
for rep in 1 2; do
  ORBX_AB_SETTINGS=frame,frame_if1 timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd32 1,2,4,8 > $OUT/ab_$rep.txt 2>&1 || { echo "AB FAILED"; tail -5 $OUT/ab_$rep.txt; exit 1; }
  cat $OUT/ab_$rep.txt
done
B=$PWD/tests/native/facade_test
LD_LIBRARY_PATH=$PWD/tools/_var/tune:$LD_LIBRARY_PATH ORBX_FS_STATS=1 timeout -k 10 120 $B bench /tmp/dd32 200 20 8 frame > $OUT/s8.json 2> $OUT/s8.err || { echo "STATS RUN FAILED"; exit 1; }
cat $OUT/s8.err
