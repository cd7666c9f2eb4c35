#!/bin/bash
# Round-4 GPU session: GPU tests, drop-in small-batch A/B, headline / bf benches, blur-stripe
# variants (timing + parity of the candidate default).  usage: tools/gpu_session_r4.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
python tools/dropin_data.py /tmp/dd 8 > /dev/null || exit 1
timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd 1,8 > $OUT/dropin_ab.txt 2>&1 || { echo "DROPIN AB FAILED"; tail -5 $OUT/dropin_ab.txt; exit 1; }
cat $OUT/dropin_ab.txt
timeout -k 10 300 python bench.py --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --workload bf --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bf.json 2> $OUT/bf.err || { echo "BF FAILED"; tail -20 $OUT/bf.err; exit 1; }
timeout -k 10 400 python tools/variants.py run > $OUT/variants.txt 2>&1 || { echo "VARIANTS FAILED"; tail -20 $OUT/variants.txt; exit 1; }
cat $OUT/variants.txt
timeout -k 10 400 bash tools/var_traffic.sh $OUT/vt base fastxcd stripe_lds3 > $OUT/var_traffic.txt 2>&1 || { echo "VAR TRAFFIC FAILED"; tail -20 $OUT/var_traffic.txt; exit 1; }
cat $OUT/var_traffic.txt
ORBX_LIB=$PWD/my_orb_slam2_amd/liborbx_stripe_lds3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_golden.py "tests/test_gpu_bench_geometry.py::test_c2_stereo_b512" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_stripe.log 2>&1 || { echo "STRIPE TESTS FAILED"; tail -30 $OUT/pytest_stripe.log; exit 1; }
tail -2 $OUT/pytest_stripe.log
echo session done
