#!/bin/bash
# k_stereo lanes-per-keypoint variants (tools/_variants.json): the stereo parity tests per
# variant, the one-call stereo Frame at K = 1 / 8, k_stereo's time at one pair (kernel trace)
# and, with "headline" as $2, the B = 512 bench per variant.  usage: TAG [headline]
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT /tmp/vl
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd 32 > /dev/null || exit 1
B=$PWD/tests/native/facade_test
for v in $(python -c "import json;print(' '.join(json.load(open('tools/_variants.json'))))"); do
  ORBX_LIB=$PWD/my_orb_slam2_amd/liborbx_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_golden.py tests/test_gpu_bench_geometry.py -m gpu -q -x -k "stereo or frame_server" --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { echo "TESTS $v FAILED"; tail -20 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
  mkdir -p /tmp/vl/$v && cp my_orb_slam2_amd/liborbx_$v.so /tmp/vl/$v/liborbx.so
  for K in 1 8; do
    F=$([ $K = 1 ] && echo 300 || echo 200)
    LD_LIBRARY_PATH=/tmp/vl/$v:$LD_LIBRARY_PATH timeout -k 10 120 $B bench /tmp/dd $F 20 $K frame > $OUT/frame_${v}_k$K.json || exit 1
    python -c "
import json; j=json.load(open('$OUT/frame_${v}_k$K.json')); v=sorted(j['latency_ms'])
print('$v K=$K median', v[len(v)//2], 'pairs/s', round(j['trackers']*j['frames']/(j['wall_ms']/1e3)), j['digests'][0])"
  done
  LD_LIBRARY_PATH=/tmp/vl/$v:$LD_LIBRARY_PATH timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/st_$v -o run -- $B bench /tmp/dd 60 10 1 frame > $OUT/st_$v.log 2>&1 || { echo "TRACE $v FAILED"; tail -3 $OUT/st_$v.log; exit 1; }
  python - $OUT/st_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_stereo' in r['Name'] or 'octree' in r['Name']: print(' ', sys.argv[2], r['Name'][:30], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
PY
done
if [ "$2" = "headline" ]; then
  timeout -k 10 700 python tools/variants.py run > $OUT/variants.txt 2>&1 || { echo "VARIANTS FAILED"; tail -20 $OUT/variants.txt; exit 1; }
  cat $OUT/variants.txt
fi
