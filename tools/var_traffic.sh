#!/bin/bash
# Per-variant FETCH_SIZE / WRITE_SIZE passes (tools/variants.py libraries), one rocprofv3 run
# per counter and variant.  usage: tools/var_traffic.sh OUT NAME...
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
for v in "$@"; do
  export ORBX_LIB=my_orb_slam2_amd/liborbx_$v.so
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/f_$v.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/w_$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing > $OUT/w_$v.log 2>&1
  echo "done $v"
done
