#!/bin/bash
# Interleaved repeats of the one-call stereo Frame (K = 1 and 8) per k_stereo variant (the
# variant libraries of tools/variants.py), to separate a small latency change from the run-order
# spread.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT /tmp/vl
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd 32 > /dev/null || exit 1
B=$PWD/tests/native/facade_test
VS=$(python -c "import json;print(' '.join(json.load(open('tools/_variants.json'))))")
for v in $VS; do mkdir -p /tmp/vl/$v && cp my_orb_slam2_amd/liborbx_$v.so /tmp/vl/$v/liborbx.so; done
for rep in 1 2 3 4; do
  for v in $VS; do
    for K in 1 8; do
      F=$([ $K = 1 ] && echo 400 || echo 200)
      LD_LIBRARY_PATH=/tmp/vl/$v:$LD_LIBRARY_PATH timeout -k 10 120 $B bench /tmp/dd $F 30 $K frame > $OUT/f_${v}_$K.json || exit 1
      python -c "
import json; j=json.load(open('$OUT/f_${v}_$K.json')); v=sorted(j['latency_ms'])
print('rep$rep $v K=$K median', v[len(v)//2], 'mean', round(sum(v)/len(v),4), 'pairs/s', round(j['trackers']*j['frames']/(j['wall_ms']/1e3)))"
    done
  done
done
