# A/B session of the built variants (tools/variants.py build ...): GPU tests on the product
# library, the headline per variant (interleaved), one-stream FETCH / WRITE passes per variant,
# the drop-in line per variant.  usage: bash tools/_ab_cmd.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python tools/variants.py run --rounds 2 --steps 50 --warmup 5 > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
for v in $(python3 -c "import json; print(' '.join(json.load(open('tools/_variants.json'))))"); do
  L=$PWD/my_orb_slam2_amd/liborbx_$v.so
  for c in FETCH_SIZE WRITE_SIZE; do
    ORBX_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${c}_$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 --no-kernel-timing --overlap 0 --inflight 1 > $O/${c}_$v.log 2>&1 || exit 1
  done
  mkdir -p /tmp/lib_$v && cp $L /tmp/lib_$v/liborbx.so
  LD_LIBRARY_PATH=/tmp/lib_$v:$LD_LIBRARY_PATH ORBX_LIB=$L timeout -k 10 300 python bench.py --workload dropin --trackers 1,8 --frames 300 --cpu-seconds 0 > $O/dropin_$v.json 2> $O/dropin_$v.err || { tail -5 $O/dropin_$v.err; exit 1; }
done
echo done
