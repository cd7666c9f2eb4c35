"""Probe: does splitting a 256-pair step into k chunks on k HIP streams overlap the
latency-bound kernels (octree, stereo) of one chunk with the issue-bound kernels of another?
usage: python tools/overlap_probe.py [B] [steps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import my_orb_slam2_amd as orbx  # noqa: E402
from my_orb_slam2_amd import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
pairs = [synth.stereo_pair(i, 1241, 376) for i in range(32)]
Lh = np.stack([pairs[i % 32][0] for i in range(B)])
Rh = np.stack([pairs[i % 32][1] for i in range(B)])
Ls, Rs = torch.from_numpy(Lh).to(dev), torch.from_numpy(Rh).to(dev)
mbf, mb = 386.1448, float(np.float32(386.1448) / np.float32(718.856))

for k in (1, 2, 4):
    n = B // k
    sbs = [orbx.StereoBatch(n, 2000, 1.2, 8, 20, 7, device=0) for _ in range(k)]
    streams = [torch.cuda.Stream(dev) for _ in range(k)]
    main = torch.cuda.current_stream(dev)

    def step():
        ev = torch.cuda.Event()
        ev.record(main)
        for i in range(k):
            streams[i].wait_event(ev)
            sbs[i](Ls[i * n:(i + 1) * n], Rs[i * n:(i + 1) * n], mbf, mb,
                   stream=streams[i].cuda_stream)
        for i in range(k):
            e = torch.cuda.Event()
            e.record(streams[i])
            main.wait_event(e)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    nv = sum(int(sb.nvalid.sum()) for sb in sbs)
    print(f"chunks={k} pairs/s={B * STEPS / dt:.0f} ms/step={1000 * dt / STEPS:.3f} nvalid={nv}",
          flush=True)
