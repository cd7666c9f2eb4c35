#!/bin/bash
# Level-0 strip height sweep (tuning build, ORBX_STRIP_TH): per height a timed bench line and
# FETCH_SIZE / WRITE_SIZE passes (each in its own rocprofv3 run).  usage: tools/l0_sweep.sh OUT LIB H...
set -e
OUT=$1; LIB=$2; shift 2
export TMPDIR=/tmp ORBX_LIB=$LIB
mkdir -p $OUT
for th in "$@"; do
  export ORBX_STRIP_TH=$th
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 > $OUT/bench_$th.json 2> $OUT/bench_$th.err
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_$th -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/f_$th.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_$th -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/w_$th.log 2>&1
  echo "done $th"
done
