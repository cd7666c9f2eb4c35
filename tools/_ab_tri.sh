# C5 triangulation: node-order database vs gather (bench.py --tri-gather), PMC FETCH / WRITE of
# each.  usage: TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "triangulation or c5 or match or boundary" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for v in gather order; do
  F=""; [ $v = gather ] && F="--tri-gather"
  timeout -k 10 300 python bench.py --workload triangulation --cpu-seconds 0 $F > $O/tri_${v}_$rep.json 2> $O/tri_${v}_$rep.err || { tail -5 $O/tri_${v}_$rep.err; exit 1; }
  python3 -c "
import json; j=json.loads(open('$O/tri_${v}_$rep.json').read().strip().splitlines()[-1]); r=j['roofline']
print('$rep $v', round(j['value']), round(r['avg_launch_ms'],4), j['mean_pairs_per_job'])"
done; done
for v in gather order; do for c in FETCH_SIZE WRITE_SIZE; do
  F=""; [ $v = gather ] && F="--tri-gather"
  timeout -s KILL 240 rocprofv3 --pmc $c -d $O/${c}_$v -o run --output-format csv -- python3 bench.py --workload triangulation --steps 3 --warmup 1 --cpu-seconds 0 $F > $O/${c}_$v.log 2>&1 || exit 1
done; done
echo done
