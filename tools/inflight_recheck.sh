#!/bin/bash
# Batches in flight re-checked on the round-6 kernels (timed schedule only, 50 steps, B = 512).
set -o pipefail
mkdir -p gpurun_out/s17
for r in 1 2; do for inf in 2 3 4; do
  timeout -k 10 200 python bench.py --inflight $inf --cpu-seconds 0 --serial-steps 0 --steps 50 > gpurun_out/s17/inf_${inf}_$r.json 2>/dev/null || { echo "FAILED $inf"; exit 1; }
  python -c "import json;j=json.loads(open('gpurun_out/s17/inf_${inf}_$r.json').read().strip().splitlines()[-1]);print($r,'inflight=$inf',round(j['value']),round(j['ms_per_step'],4),j['verified'])"
done; done
