#!/bin/bash
# Quick check on the GPU box: default bench, two / one batches in flight, drop-in, host-io and EuRoC lines.
# usage: tools/check_session.sh [OUTDIR]
set -o pipefail
O=gpurun_out/${1:-check}; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cat $O/bench.json | python -c "import json,sys; j=json.loads(sys.stdin.read()); r=j['roofline']; print('default', round(j['value']), j['ms_per_step'], r['frac'], r['avg_launch_ms'], j['one_stream'], r.get('serial_pass',{}).get('frac'), j['cpu_baseline']['value'])"
timeout -k 10 300 python tools/overlap_ab.py "3,3,1" "0" -- --steps 60 --inflight 2 > $O/inflight.txt 2>&1 || { echo INFLIGHT FAILED; cat $O/inflight.txt; exit 1; }
cat $O/inflight.txt
timeout -k 10 300 python bench.py --workload dropin --frames 300 > $O/dropin.json 2> $O/dropin.err || { echo DROPIN FAILED; tail $O/dropin.err; exit 1; }
cut -c1-600 $O/dropin.json
timeout -k 10 300 python bench.py --host-io --steps 20 --warmup 4 --cpu-seconds 0 > $O/hostio.json 2> $O/hostio.err || { echo HOSTIO FAILED; tail $O/hostio.err; exit 1; }
cut -c1-400 $O/hostio.json
timeout -k 10 300 python bench.py --workload euroc --cpu-seconds 0 > $O/euroc.json 2> $O/euroc.err || { echo EUROC FAILED; tail $O/euroc.err; exit 1; }
cut -c1-300 $O/euroc.json
