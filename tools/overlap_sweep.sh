#!/bin/bash
# overlap sweep (B = 512), two rounds interleaved
set -o pipefail
OUT=gpurun_out/r5ovl
mkdir -p $OUT
for rep in 1 2; do
for ov in 3,3,1 3,2,1 3,4,1 2,3,1 3,3,2 3,5,1; do
  timeout -k 10 200 python bench.py --overlap $ov --steps 60 --warmup 10 --cpu-seconds 0 --serial-steps 0 > $OUT/b_${ov}_$rep.json 2> $OUT/b_${ov}_$rep.err || { echo "FAILED $ov"; tail -5 $OUT/b_${ov}_$rep.err; exit 1; }
  python -c "import json; j=json.loads(open('$OUT/b_${ov}_$rep.json').read().strip().splitlines()[-1]); print('$ov', $rep, round(j['value']), round(j['ms_per_step'],4))"
done
done
