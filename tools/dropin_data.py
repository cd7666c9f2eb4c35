"""Writes the drop-in bench's input directory (bench.py --workload dropin) for running
tests/native/boundary_test `bench` directly, e.g. under rocprofv3:
    python tools/dropin_data.py DIR [P]
    rocprofv3 --kernel-trace --stats -d OUT -o run -- tests/native/boundary_test bench DIR 200 20 K
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

d = sys.argv[1]
P = int(sys.argv[2]) if len(sys.argv) > 2 else 32
os.makedirs(d, exist_ok=True)
Lh, Rh, _, _ = bench.stereo_inputs(0, P, P)
for i in range(P):
    Lh[i].tofile(os.path.join(d, f"pair_{i}_left.raw"))
    Rh[i].tofile(os.path.join(d, f"pair_{i}_right.raw"))
mb = float(np.float32(bench.MBF) / np.float32(bench.FX))
with open(os.path.join(d, "params.txt"), "w") as f:
    f.write(f"{bench.W} {bench.H} {bench.NFEAT} {bench.MBF!r} {mb!r} {P}\n")
print(d)
