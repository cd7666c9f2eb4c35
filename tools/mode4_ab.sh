#!/bin/bash
# Mode 4 (level 0's blur on the side branch) against mode 3, two batches and one batch in flight.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 200 --timeout-method thread -k "overlap or graph" > $O/pytest.log 2>&1 || { echo TEST FAILED; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "inflight 2" >> $O/ab.txt
  timeout -k 10 400 python tools/overlap_ab.py "3,3,1" "4,1,1" "4,2,1" "4,3,1" -- --steps 60 >> $O/ab.txt 2>&1 || { echo AB FAILED; cat $O/ab.txt; exit 1; }
  echo "inflight 1" >> $O/ab.txt
  timeout -k 10 400 python tools/overlap_ab.py "3,3,1" "4,1,1" "4,3,1" -- --steps 60 --inflight 1 >> $O/ab.txt 2>&1 || { echo AB FAILED; cat $O/ab.txt; exit 1; }
done
cat $O/ab.txt
