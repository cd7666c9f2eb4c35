"""Diagnostic: per-phase clocks of k_pyr_chain for one image (separate -DORBX_CHAIN_STAMPS
build; never quote its run time).  usage: python tools/chain_stamps.py [build]"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from my_orb_slam2_amd import build as b  # noqa: E402

VAR = int(os.environ.get("CHAIN_DIAG", "0"))   # CHAIN_DIAG variant of the diagnostic build
DIAG = os.path.join(ROOT, "tools", "_diag", f"liborbx_chaindiag{VAR}.so")
os.makedirs(os.path.dirname(DIAG), exist_ok=True)
srcs = [str(b.CSRC / s) for s in b.SOURCES if (b.CSRC / s).exists()]
newest = max(os.path.getmtime(str(b.CSRC / f)) for f in os.listdir(b.CSRC))
if not os.path.exists(DIAG) or os.path.getmtime(DIAG) < newest:
    subprocess.run([b.hipcc()] + b.FLAGS + ["-DORBX_CHAIN_STAMPS", f"-DCHAIN_DIAG={VAR}"] + srcs + ["-o", DIAG], check=True)
if len(sys.argv) > 1 and sys.argv[1] == "build":
    sys.exit(0)
import torch  # noqa: E402,F401
from my_orb_slam2_amd import _lib, synth  # noqa: E402
_lib._lib = _lib.load(DIAG)
import my_orb_slam2_amd as m  # noqa: E402

img = synth.stereo_pair(0)[0]
ext = m.ORBextractor(2000, 1.2, 8, 20, 7)
for _ in range(5):
    ext(img)
st = np.zeros((256, 40), np.uint64)
_lib._lib.orbx_diag_chain_stamps(ctypes.c_void_p(st.ctypes.data))
t0 = st[st[:, 0] > 0, 0].min()
for t in range(0, 64, 9):
    s = st[t].astype(np.int64)
    if s[0] == 0:
        continue
    marks = [int(v - s[0]) if v else -1 for v in s[:19]]
    print(f"tile {t:3d}  " + " ".join(f"{x:6d}" for x in marks))
    # per level l >= 1: [columns of l-1 done, own resize items done, barrier passed, rows done]
    print("          " + "  ".join(f"L{l}:{int(s[18 + 2 * l] - s[0])}/{int(s[19 + 2 * l] - s[0])}/{int(s[2 + 2 * l] - s[0])}/{int(s[3 + 2 * l] - s[0])}" for l in range(1, 8) if 19 + 2 * l < 40))
ends = st[:, 18].astype(np.int64)
print("last end (cycles from first start):", int(ends[ends > 0].max() - t0))
