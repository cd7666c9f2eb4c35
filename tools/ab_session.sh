#!/bin/bash
# A/B session on the GPU box: the GPU tests on the product library, then bench.py once per
# side-branch configuration (tools/overlap_ab.py), twice over.
# usage: tools/ab_session.sh OUTDIR "cfg cfg ..." [bench args]
set -o pipefail
O=gpurun_out/$1; shift
CF=$1; shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 600 python tools/overlap_ab.py $CF -- --steps 60 "$@" >> $O/ab.txt 2>&1 || { echo "AB FAILED"; cat $O/ab.txt; exit 1; }
done
cat $O/ab.txt
