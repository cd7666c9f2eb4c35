#!/bin/bash
# Batches in flight x side branch (B=512, 60 timed steps), twice over.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for rep in 1 2; do
  for nf in 1 2 3; do
    echo "inflight $nf" >> $O/ab.txt
    timeout -k 10 300 python tools/overlap_ab.py "0" "3,3,1" "3,3,2" -- --steps 60 --inflight $nf >> $O/ab.txt 2>&1 || { echo AB FAILED; cat $O/ab.txt; exit 1; }
  done
  echo "inflight 1, fork after the last level" >> $O/ab.txt
  timeout -k 10 300 python tools/overlap_ab.py "3,8,1" -- --steps 60 >> $O/ab.txt 2>&1 || { echo AB FAILED; cat $O/ab.txt; exit 1; }
done
timeout -k 10 300 python bench.py --host-io --steps 20 --warmup 4 --cpu-seconds 0 > $O/hostio.json 2> $O/hostio.err || { echo HOSTIO FAILED; tail $O/hostio.err; exit 1; }
python -c "import json; j=json.load(open('$O/hostio.json')); print('hostio', round(j['value']), j['pcie_bound_frac'])" >> $O/ab.txt
cat $O/ab.txt
