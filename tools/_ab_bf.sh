# BF A/B: parity tests, then bench.py --workload bf per built variant (interleaved) and
# FETCH / WRITE passes per variant.  usage: TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bf.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
V=$(python3 -c "import json; print(' '.join(json.load(open('tools/_variants.json'))))")
for rep in 1 2; do for v in $V; do
  ORBX_LIB=$PWD/my_orb_slam2_amd/liborbx_$v.so timeout -k 10 300 python bench.py --workload bf --steps 20 --warmup 3 --cpu-seconds 0 > $O/bf_${v}_$rep.json 2> $O/bf_${v}_$rep.err || { tail -5 $O/bf_${v}_$rep.err; exit 1; }
  python3 -c "
import json; j=json.loads(open('$O/bf_${v}_$rep.json').read().strip().splitlines()[-1]); r=j['roofline']; a=j['alt_kernel']
print('$rep $v', round(j['value'],1), round(r['avg_launch_ms'],3), round(r['frac'],3), j['planted_found'], '| alt', a['kernel'], round(a['value'],1), a['outputs_equal_default'])"
done; done
for v in $V; do for c in FETCH_SIZE WRITE_SIZE; do
  ORBX_LIB=$PWD/my_orb_slam2_amd/liborbx_$v.so timeout -s KILL 240 rocprofv3 --pmc $c -d $O/${c}_$v -o run --output-format csv -- python3 bench.py --workload bf --steps 3 --warmup 1 --cpu-seconds 0 > $O/${c}_$v.log 2>&1 || exit 1
done; done
echo done
