#!/bin/bash
# stereo hand-off variants (tools/stereo_ab.sh), then the drop-in A/B with the side branch in
# the stereo-frame graph.  usage: TAG
set -o pipefail
bash tools/stereo_ab.sh $1 || exit 1
OUT=gpurun_out/$1
timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd 1,8 > $OUT/dropin_ab.txt 2>&1 || { echo "DROPIN AB FAILED"; tail -5 $OUT/dropin_ab.txt; exit 1; }
grep frame $OUT/dropin_ab.txt
