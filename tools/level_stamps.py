"""Diagnostic: phase shares of k_level from s_memtime stamps (separate -DORBX_STAMPS build;
never quote its run time).  usage: python tools/level_stamps.py"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from my_orb_slam2_amd import build as b  # noqa: E402

DIAG = os.path.join(ROOT, "tools", "_diag", "liborbx_diag.so")
os.makedirs(os.path.dirname(DIAG), exist_ok=True)
srcs = [str(b.CSRC / s) for s in b.SOURCES if (b.CSRC / s).exists()]
newest = max(os.path.getmtime(str(b.CSRC / f)) for f in os.listdir(b.CSRC))
if not os.path.exists(DIAG) or os.path.getmtime(DIAG) < newest:
    subprocess.run([b.hipcc()] + b.FLAGS + ["-DORBX_STAMPS"] + srcs + ["-o", DIAG], check=True)
if len(sys.argv) > 1 and sys.argv[1] == "build":
    sys.exit(0)
import torch  # noqa: E402
from my_orb_slam2_amd import _lib, synth  # noqa: E402
_lib._lib = _lib.load(DIAG)
import my_orb_slam2_amd as m  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pairs = [synth.stereo_pair(i) for i in range(4)]
L = torch.from_numpy(np.stack([pairs[i % 4][0] for i in range(B)])).cuda()
R = torch.from_numpy(np.stack([pairs[i % 4][1] for i in range(B)])).cuda()
sb = m.StereoBatch(B, 2000, 1.2, 8, 20, 7)
mb = float(np.float32(386.1448) / np.float32(718.856))
for _ in range(3):
    sb(L, R, 386.1448, mb)
torch.cuda.synchronize()
st = np.zeros((8, 4096, 6), np.uint64)
_lib._lib.orbx_diag_level_stamps(ctypes.c_void_p(st.ctypes.data))
names = ["stage+tables", "level", "out+rows", "columns"]
for l in range(8):
    s = st[l].astype(np.int64)
    ok = (s[:, 0] > 0) & (s[:, 5] > s[:, 0])
    d = np.diff(s[ok][:, [0, 2, 3, 4, 5]], axis=1)
    tot = d.sum(1)
    print(f"L{l} blocks {ok.sum():5d} mean cycles {tot.mean():8.0f}  " +
          "  ".join(f"{n} {100 * d[:, i].sum() / tot.sum():4.1f}%" for i, n in enumerate(names)))
