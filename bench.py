#!/usr/bin/env python3
"""Throughput benchmark of the ORB stereo front-end (BASELINE.json metric).

Workload (BASELINE.json configs[1]): KITTI-size 1241x376 rectified stereo pairs, 2000
features per image; one step = ORBextractor on B left + B right images and
Frame::ComputeStereoMatches on the B pairs, inputs resident in HBM before timing.
Synthetic frames (no datasets in the image): my_orb_slam2_amd.synth.stereo_pair.

    python bench.py [--gpus N --steps K --warmup W --batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank/GPU)

Multi-GPU: pairs are independent (src/Frame.cc:72-130), so every rank runs its own batch
with no collective in the data path (weak scaling); only the timing uses a barrier and a
max-reduction.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match, KITTI 1241×376 stereo, 1/2/4/8 GPU"
W, H, NFEAT = 1241, 376, 2000
MBF, FX = 386.1448, 718.856            # Examples/Stereo/KITTI00-02.yaml:8,25
HBM_PEAK_GBS = 8000.0                  # MI355X_MICROARCH.md: 8 TB/s spec


HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_PMC = ",".join(os.path.join(HERE, "profiles", f) for f in
                       ("r01_pmc_fetch_b256.csv", "r01_pmc_write_b256.csv"))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="stereo pairs per step per GPU")
    ap.add_argument("--distinct", type=int, default=32, help="distinct synthetic pairs")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU-baseline sample budget (0 disables)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--traffic-csv", default=DEFAULT_PMC,
                    help="comma-separated rocprofv3 --pmc counter CSVs (globs) holding FETCH_SIZE"
                         " and WRITE_SIZE for the roofline traffic field (default: the"
                         " committed profiles/ summaries of this workload)")
    return ap.parse_args()


def algorithmic_bytes_fast(level_sizes, cells_area_read, ncand):
    """k_fast: every cell ROI byte read once + one count and 4 B per candidate written."""
    return cells_area_read + 4 * ncand


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import my_orb_slam2_amd as orbx
    from my_orb_slam2_amd import synth

    B = args.batch
    P = max(1, min(args.distinct, B))
    pairs = [synth.stereo_pair(1000 * rank + i, W, H) for i in range(P)]
    idx = [i % P for i in range(B)]
    Lh = np.stack([pairs[i][0] for i in idx])
    Rh = np.stack([pairs[i][1] for i in idx])
    Ls = torch.from_numpy(Lh).to(dev)
    Rs = torch.from_numpy(Rh).to(dev)
    torch.cuda.synchronize(dev)

    mb = float(np.float32(MBF) / np.float32(FX))
    sb = orbx.StereoBatch(B, NFEAT, 1.2, 8, 20, 7, device=local)
    stream = torch.cuda.current_stream(dev)
    st = stream.cuda_stream

    for _ in range(args.warmup):
        sb(Ls, Rs, MBF, mb, stream=st)
    torch.cuda.synchronize(dev)
    if not args.no_kernel_timing:
        sb.profile(True)
        sb.collect_profile()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sb(Ls, Rs, MBF, mb, stream=st)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    prof = sb.collect_profile() if not args.no_kernel_timing else {}

    # sanity on the produced work (outside the timed region)
    nv = sb.nvalid.cpu().numpy()
    nkp, _, _ = sb.fetch("left")

    total_pairs = B * args.steps * world
    fps = total_pairs / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # roofline of the dominant kernel
    roof = None
    if prof:
        dom = max(prof, key=lambda k: prof[k][0])
        tot_ms, launches = prof[dom]
        avg_s = tot_ms / 1000.0 / max(launches, 1)
        geo = kernel_bytes(sb, B)
        alg = geo.get(dom)
        achieved = (alg / avg_s / 1e9) if (alg and avg_s > 0) else None
        roof = {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic_from_csv(args.traffic_csv, dom),
                "algorithmic_bytes_per_launch": alg, "avg_launch_ms": avg_s * 1000.0,
                "kernel_ms_per_step": {k: round(v[0] / max(args.steps, 1), 4)
                                       for k, v in prof.items()}}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(pairs, mb, args.cpu_seconds)

    if rank == 0:
        out = {"metric": METRIC, "value": fps, "unit": "frames/sec", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "u8", "data": "synthetic",
               "config": {"workload": "kitti_stereo_extract_match", "width": W, "height": H,
                          "nfeatures": NFEAT, "nlevels": 8, "scale_factor": 1.2,
                          "pairs_per_step_per_gpu": B, "distinct_pairs": P,
                          "parallelism": f"dp{world}"},
               "mean_keypoints_left": float(nkp.mean()),
               "mean_stereo_matches": float(nv.mean()),
               "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def kernel_bytes(sb, B):
    """Algorithmic HBM bytes per launch of each kernel.  One launch
    covers the 2B views (k_level: one level of them)."""
    v = sb.ext.batch_view()
    L = 8
    area = [v.level_w[l] * v.level_h[l] for l in range(L)]
    n = 2 * B
    kc = v.kp_cap
    return {
        # per level: read level l-1 (level 0: the input), write level l and its blur
        "k_level": n * (sum(area[:-1]) + area[0] + 2 * sum(area)) / L,
        # every level byte read once
        "k_fast": n * sum(area),
        # candidates in (<= 4 B each, bounded by 2 x kp slots here) and survivors out
        "k_octree": n * 4 * kc * 2,
        # 31x31 raw + 37x37 blurred patch in, 28 + 32 B out per keypoint
        "k_orient_desc": n * kc * (31 * 31 + 37 * 37 + 60),
        # both views' keypoints + descriptors in, 11x11 + 11x21 SAD windows, 8 B out
        "k_stereo": B * kc * (2 * (28 + 32) + 11 * 11 + 11 * 21 + 8),
    }


def traffic_from_csv(paths, kernel):
    """HBM bytes per launch of `kernel` from rocprofv3 --pmc counter CSVs (FETCH_SIZE and
    WRITE_SIZE come from separate passes, MI355X_MICROARCH.md §HBM): each counter is
    averaged over the kernel's dispatches in the file that holds it; both are KiB; FETCH_SIZE
    is doubled (gfx950 tallies a wide streaming read at half its bytes)."""
    import csv
    import glob
    files = []
    for p in (paths or "").split(","):
        files += sorted(glob.glob(p.strip())) if p.strip() else []
    per = {}
    for path in files:
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                name = row.get("Counter_Name")
                if name in ("FETCH_SIZE", "WRITE_SIZE"):
                    tot, ids = per.setdefault(name, [0.0, set()])
                    per[name][0] = tot + float(row["Counter_Value"])
                    ids.add((path, row.get("Dispatch_Id")))
    if "FETCH_SIZE" not in per or "WRITE_SIZE" not in per:
        return None
    fetch = per["FETCH_SIZE"][0] / len(per["FETCH_SIZE"][1])
    write = per["WRITE_SIZE"][0] / len(per["WRITE_SIZE"][1])
    return (2.0 * fetch + write) * 1024.0


def cpu_baseline(pairs, mb, budget_s):
    """The CPU restatement timed on this host: reference-faithful mode (src/Frame.cc:89-102:
    left and right extraction on two threads, then ComputeStereoMatches on one)."""
    try:
        import oracle
    except Exception:
        return None
    ol = oracle.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
    orr = oracle.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
    done = 0
    t0 = time.perf_counter()
    while True:
        Lp, Rp = pairs[done % len(pairs)]
        res = {}
        th = threading.Thread(target=lambda: res.__setitem__("r", orr(Rp)))
        th.start()
        kl, _ = ol(Lp)
        th.join()
        oracle.stereo_match(ol, orr, len(kl), MBF, mb)
        done += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    el = time.perf_counter() - t0
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": done / el, "unit": "frames/sec", "cores": 2, "kind": "port",
            "sample": f"{done} KITTI-size synthetic stereo pairs, L/R extraction on 2 threads + "
                      f"ComputeStereoMatches (Frame.cc:89-102), {el:.1f} s",
            "cpu_model": model, "host_cpus": os.cpu_count()}


if __name__ == "__main__":
    main()
