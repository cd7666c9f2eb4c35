"""Diagnostic: phase cycles of k_fast from s_memtime stamps (separate -DORBX_STAMPS build;
never quote its run time).  usage: python tools/fast_stamps.py [B]"""
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
newest = max(os.path.getmtime(p) for p in srcs + [str(b.CSRC / h) for h in os.listdir(b.CSRC)])
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
st = np.zeros((16384, 8), np.uint64)
_lib._lib.orbx_diag_fast_stamps(ctypes.c_void_p(st.ctypes.data))
s = st.astype(np.int64)
ok = s[:, 4] > 0
s = s[ok]
tot = s[:, 4].sum()
names = ["stage+zero", "compass+list", "arc score", "nms+out"]
print(f"cells {ok.sum()}  mean cycles/wave {s[:, 4].mean():.0f}  " +
      "  ".join(f"{n} {100 * s[:, i].sum() / tot:4.1f}%" for i, n in enumerate(names)))
print(f"survivors/px {s[:, 5].sum() / s[:, 7].sum():.3f}  corners/px {s[:, 6].sum() / s[:, 7].sum():.4f}"
      f"  px/cell {s[:, 7].mean():.0f}")
for lo, hi in [(0, 400), (400, 800), (800, 1200), (1200, 5000)]:
    sel = (s[:, 7] >= lo) & (s[:, 7] < hi)
    if sel.any():
        print(f"  px in [{lo},{hi}): cells {sel.sum():5d} cycles {s[sel, 4].mean():7.0f} "
              f"surv/px {s[sel, 5].sum() / max(s[sel, 7].sum(), 1):.3f}")
