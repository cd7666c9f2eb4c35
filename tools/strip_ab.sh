#!/bin/bash
# A/B of per-level strip heights at B = 512 (tuning build, ORBX_STRIP_TH), interleaved:
# one-stream levels 1-7 and the timed step.  usage: tools/strip_ab.sh TAG "h0,h1,..." ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
LIB=$PWD/tools/_var/tune/liborbx.so
for rep in 1 2; do
  i=0
  for th in default "$@"; do
    i=$((i+1))
    if [ "$th" = default ]; then envs=""; else envs="ORBX_STRIP_TH=$th"; fi
    env ORBX_LIB=$LIB $envs timeout -k 10 200 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 > $OUT/s${i}_$rep.json 2> $OUT/s${i}_$rep.err || { echo "FAILED $th"; tail -5 $OUT/s${i}_$rep.err; exit 1; }
    python -c "import json; j=json.loads(open('$OUT/s${i}_$rep.json').read().strip().splitlines()[-1]); r=j['roofline']['one_stream_ms_per_step']; print('$th', $rep, round(j['value']), round(j['ms_per_step'],4), 'L0', r['k_level0'], 'L1-7', r['k_level1_7'])"
  done
done
