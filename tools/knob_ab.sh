#!/bin/bash
# Compile-time knob variants (tools/variants.py build ...) timed in the default schedule.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 600 python tools/variants.py run --steps 60 >> $O/ab.txt 2>&1 || { echo AB FAILED; cat $O/ab.txt; exit 1; }
done
cat $O/ab.txt
