#!/bin/bash
# The one-call stereo Frame (facade_test bench ... frame): HIP API + kernel + copy traces at
# K = 1 and K = 8.  usage: tools/frame_trace.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd 8 > /dev/null || exit 1
B=tests/native/facade_test
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr1 -o run -- $B bench /tmp/dd 60 10 1 frame > $OUT/tr1.log 2>&1 || { echo "TRACE K=1 FAILED"; tail -5 $OUT/tr1.log; exit 1; }
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr8 -o run -- $B bench /tmp/dd 30 10 8 frame > $OUT/tr8.log 2>&1 || { echo "TRACE K=8 FAILED"; tail -5 $OUT/tr8.log; exit 1; }
echo done
