"""Diagnostic: per-round clocks of k_octree for one image of a stereo batch (separate
-DORBX_OCT_STAMPS build; never quote its run time).  usage: python tools/octree_stamps.py [B]"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from my_orb_slam2_amd import build as b  # noqa: E402

IMG = int(os.environ.get("OCT_STAMP_IMG", "5"))   # blockIdx.y whose lists are stamped
DIAG = os.path.join(ROOT, "tools", "_diag", f"liborbx_octdiag{IMG}.so")
os.makedirs(os.path.dirname(DIAG), exist_ok=True)
srcs = [str(b.CSRC / s) for s in b.SOURCES if (b.CSRC / s).exists()]
newest = max(os.path.getmtime(str(b.CSRC / f)) for f in os.listdir(b.CSRC))
if not os.path.exists(DIAG) or os.path.getmtime(DIAG) < newest:
    subprocess.run([b.hipcc()] + b.FLAGS + [f"-DORBX_OCT_STAMPS={IMG}"] + srcs + ["-o", DIAG], check=True)
if len(sys.argv) > 1 and sys.argv[1] == "build":
    sys.exit(0)
import torch  # noqa: E402
from my_orb_slam2_amd import _lib, synth  # noqa: E402
_lib._lib = _lib.load(DIAG)
import my_orb_slam2_amd as m  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
pairs = [synth.stereo_pair(i) for i in range(4)]
L = torch.from_numpy(np.stack([pairs[i % 4][0] for i in range(B)])).cuda()
R = torch.from_numpy(np.stack([pairs[i % 4][1] for i in range(B)])).cuda()
sb = m.StereoBatch(B, 2000, 1.2, 8, 20, 7)
mb = float(np.float32(386.1448) / np.float32(718.856))
for _ in range(3):
    sb(L, R, 386.1448, mb)
torch.cuda.synchronize()
st = np.zeros((16, 64), np.uint64)
_lib._lib.orbx_diag_octree_stamps(ctypes.c_void_p(st.ctypes.data))
for lv in range(8):
    s = st[lv].astype(np.int64)
    t0 = s[0]
    tot = s[61] - t0
    rounds = []
    for g in range(28):
        a, e = s[3 + 2 * g], s[4 + 2 * g]
        if a == 0 or e == 0:
            break
        rounds.append(e - a)
    print(f"L{lv} total {tot:8d} cyc  gather {s[1] - t0:7d}  roots {s[2] - s[1]:6d}  "
          f"rounds {len(rounds)}: {rounds}  final {s[61] - s[60]:6d}")
