#!/bin/bash
# Drop-in stereo diagnosis: boundary_test `run` on the KITTI fixture pair with the product
# library, without the extraction graph, and with the two-launch stereo cut.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT /tmp/ds/lib
export TMPDIR=/tmp
python - <<'PY' || exit 1
import json, pathlib, numpy as np, sys
sys.path.insert(0, '.')
from my_orb_slam2_amd import synth
g = json.load(open('tests/golden/fixtures.json'))['kitti_stereo_seed0']
L, R = synth.stereo_pair(0)
d = pathlib.Path('/tmp/ds'); H, W = L.shape
(d / 'left.raw').write_bytes(L.tobytes()); (d / 'right.raw').write_bytes(R.tobytes())
F12 = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32)
(d / 'params.txt').write_text(f"{W} {H} {g['params'][0]} {g['mbf']!r} {g['mb']!r} 10000000.0 0.0 " +
                              " ".join(repr(float(v)) for v in F12.reshape(-1)))
print('golden n_valid', g['n_valid'])
PY
timeout -k 10 60 tests/native/boundary_test run /tmp/ds > $OUT/default.txt 2>&1; echo "default rc=$?"; cat $OUT/default.txt
ORBX_EXTRACT_GRAPH=0 timeout -k 10 60 tests/native/boundary_test run /tmp/ds > $OUT/nograph.txt 2>&1; echo "nograph rc=$?"; cat $OUT/nograph.txt
cp my_orb_slam2_amd/liborbx_nofuse.so /tmp/ds/lib/liborbx.so
LD_LIBRARY_PATH=/tmp/ds/lib:$LD_LIBRARY_PATH timeout -k 10 60 tests/native/boundary_test run /tmp/ds > $OUT/nofuse.txt 2>&1; echo "nofuse rc=$?"; cat $OUT/nofuse.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "stereo" > $OUT/pytest_stereo.log 2>&1; echo "pytest stereo rc=$?"; tail -15 $OUT/pytest_stereo.log
