#!/bin/bash
# GPU tests, then the drop-in and TUM per-frame latency lines (orbx_extract's graph path).
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload dropin --frames 300 > $O/dropin_$rep.json 2> $O/dropin.err || { echo DROPIN FAILED; tail $O/dropin.err; exit 1; }
  timeout -k 10 300 python bench.py --workload tum --frames 300 > $O/tum_$rep.json 2> $O/tum.err || { echo TUM FAILED; tail $O/tum.err; exit 1; }
  python -c "import json; a=json.load(open('$O/dropin_$rep.json'))['latency']; b=json.load(open('$O/tum_$rep.json'))['latency']; print('dropin median/mean', round(a['median_ms'],4), round(a['mean_ms'],4), 'tum median/mean', round(b['median_ms'],4), round(b['mean_ms'],4))"
done
