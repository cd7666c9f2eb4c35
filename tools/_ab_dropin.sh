# Interleaved drop-in A/B of the built variants (K = 1 and 8, two rounds).  usage: TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
V=$(python3 -c "import json; print(' '.join(json.load(open('tools/_variants.json'))))")
for v in $V; do mkdir -p /tmp/lib_$v && cp my_orb_slam2_amd/liborbx_$v.so /tmp/lib_$v/liborbx.so; done
for rep in 1 2; do
  for v in $V; do
    LD_LIBRARY_PATH=/tmp/lib_$v:$LD_LIBRARY_PATH timeout -k 10 300 python bench.py --workload dropin --trackers 1,8 --frames 400 --cpu-seconds 0 > $O/dropin_${v}_$rep.json 2> $O/dropin_${v}_$rep.err || { tail -5 $O/dropin_${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/dropin_${v}_$rep.json').read().strip().splitlines()[-1])
print('$rep $v', [(p['trackers'], p['latency']['median_ms'], round(p['pairs_per_s'])) for p in d['per_trackers']], 'facade', [(p['trackers'], p['latency']['median_ms']) for p in d['two_thread_facade']['per_trackers']])"
  done
done
