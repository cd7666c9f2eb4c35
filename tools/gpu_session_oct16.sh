#!/bin/bash
# The octree's small-batch LDS budget for frame-server batches (up to 16 images): default
# (batches of at most 4 images) vs 16, K = 4 / 8 interleaved, then the K = 8 kernel trace of
# each.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
python tools/dropin_data.py /tmp/dd32 32 > /dev/null || exit 1
for rep in 1 2; do
  ORBX_AB_SETTINGS=frame,frame_oct16 timeout -k 10 300 python tools/dropin_ab.py run /tmp/dd32 4,8 > $OUT/ab_$rep.txt 2>&1 || { echo "AB FAILED"; tail -5 $OUT/ab_$rep.txt; exit 1; }
  cat $OUT/ab_$rep.txt
done
B=$PWD/tests/native/facade_test
for v in 4 16; do
  LD_LIBRARY_PATH=$PWD/tools/_var/tune:$LD_LIBRARY_PATH ORBX_OCT_SMALL_BATCH=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k$v -o run -- $B bench /tmp/dd32 60 10 8 frame > $OUT/k$v.log 2>&1 || { echo "TRACE FAILED"; exit 1; }
  python - $OUT/k$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'octree' in r['Name']: print('oct_small_batch', sys.argv[2], r['Name'][:30], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
done
