#!/bin/bash
# k_stereo variants (tools/_variants.json): stereo parity tests per variant, the headline bench
# per variant, and the one-call stereo Frame at K = 1 with each variant.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT /tmp/vl
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd 8 > /dev/null || exit 1
for v in $(python -c "import json;print(' '.join(json.load(open('tools/_variants.json'))))"); do
  ORBX_LIB=$PWD/my_orb_slam2_amd/liborbx_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_golden.py -m gpu -q -x -k stereo --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { echo "TESTS $v FAILED"; tail -20 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
  mkdir -p /tmp/vl/$v && cp my_orb_slam2_amd/liborbx_$v.so /tmp/vl/$v/liborbx.so
  for K in 1 8; do
    F=$([ $K = 1 ] && echo 200 || echo 100)
    LD_LIBRARY_PATH=/tmp/vl/$v:$LD_LIBRARY_PATH timeout -k 10 120 tests/native/facade_test bench /tmp/dd $F 20 $K frame > $OUT/frame_${v}_k$K.json || exit 1
    python -c "
import json; j=json.load(open('$OUT/frame_${v}_k$K.json')); v=sorted(j['latency_ms'])
print('$v K=$K median', v[len(v)//2], 'pairs/s', round(j['trackers']*j['frames']/(j['wall_ms']/1e3)), j['digests'][0])"
  done
done
if [ "$2" = "headline" ]; then
  timeout -k 10 600 python tools/variants.py run > $OUT/variants.txt 2>&1 || { echo "VARIANTS FAILED"; tail -20 $OUT/variants.txt; exit 1; }
  cat $OUT/variants.txt
fi
