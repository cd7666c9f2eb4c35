#!/bin/bash
# C4 brute-force top-2: parity tests, then the bf bench per variant (tools/_variants.json).
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bf.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in mfma xorpop; do
  ORBX_LIB=$PWD/my_orb_slam2_amd/liborbx_$v.so timeout -k 10 300 python bench.py --workload bf --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bf_$v.json 2> $OUT/bf_$v.err || { echo "BF $v FAILED"; tail -20 $OUT/bf_$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/bf_$v.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v',round(d['value'],1),d['ms_per_step'],r.get('avg_launch_ms'),r.get('issue_frac'),r.get('distances_per_s'))"
done
