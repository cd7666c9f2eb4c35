set -o pipefail
O=gpurun_out/v1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for v in bs1 s2a0; do
  ORBX_LIB=$PWD/my_orb_slam2_amd/liborbx_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_bench_geometry.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "VARIANT $v TESTS FAILED"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
timeout -k 10 600 python tools/variants.py run --steps 60 > $O/ab.txt 2>&1 || { echo "AB FAILED"; cat $O/ab.txt; exit 1; }
cat $O/ab.txt
