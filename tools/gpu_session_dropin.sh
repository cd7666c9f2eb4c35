#!/bin/bash
# Drop-in path session: its parity tests, then the small-batch A/B (tools/dropin_ab.py).
# usage: tools/gpu_session_dropin.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_golden.py tests/test_facade_cpp.py tests/test_boundary_cpp.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
python tools/dropin_data.py /tmp/dd 8 > /dev/null || exit 1
timeout -k 10 400 python tools/dropin_ab.py run /tmp/dd 1,8 > $OUT/dropin_ab.txt 2>&1 || { echo "DROPIN AB FAILED"; tail -5 $OUT/dropin_ab.txt; exit 1; }
cat $OUT/dropin_ab.txt
