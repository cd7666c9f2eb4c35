#!/bin/bash
# Frame server batches in flight: 1 / 2 (default) / 3, interleaved twice, 32 cold pairs.
# usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd32 32 > /dev/null || exit 1
for rep in 1 2; do
  ORBX_AB_SETTINGS=frame_if1,frame,frame_if3 timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd32 2,4,8 > $OUT/ab_$rep.txt 2>&1 || { echo "AB FAILED"; tail -5 $OUT/ab_$rep.txt; exit 1; }
  cat $OUT/ab_$rep.txt
done
