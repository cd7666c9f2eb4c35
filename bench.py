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
                       ("r06_pmc_fetch_b512.csv", "r06_pmc_write_b512.csv"))
DEFAULT_PMC_EUROC = ",".join(os.path.join(HERE, "profiles", f) for f in
                             ("r05_pmc_fetch_euroc.csv", "r05_pmc_write_euroc.csv"))
# FETCH_SIZE / WRITE_SIZE passes of the matcher workloads (tools/session.sh counters_match)
DEFAULT_PMC_BY_WORKLOAD = {
    "stereo": DEFAULT_PMC,
    **{w: ",".join(os.path.join(HERE, "profiles", f"r06_pmc_{c}_{w}.csv") for c in ("fetch", "write"))
       for w in ("bf", "reloc", "triangulation")}}
# SQ_INSTS_VALU and SQ_ACTIVE_INST_VALU passes (the VALU issue entry beside the HBM roofline)
DEFAULT_INSTS = ",".join(os.path.join(HERE, "profiles", f) for f in
                         ("r06_pmc_insts_b512.csv", "r06_pmc_busy_b512.csv"))
DEFAULT_INSTS_EUROC = ",".join(os.path.join(HERE, "profiles", f) for f in
                               ("r05_pmc_insts_euroc.csv", "r05_pmc_busy_euroc.csv"))
# VALU issue peaks of the chip (256 CUs x 4 SIMDs at 2.4 GHz): one wave64 instruction per
# 2 cycles per SIMD for the full-rate class (add / logic / shifts / f32 mul-add), per 4 cycles
# for the rest (v_dot*, v_perm, v_pk_*, v_bcnt, 32-bit min / max, conversions), measured by
# tools/valu_rates.hip (profiles/r01_valu_issue_rates.txt)
VALU_PEAK_2CYC = 1024 * 2.4e9 / 2
VALU_PEAK_4CYC = 1024 * 2.4e9 / 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None,
                    help="stereo pairs (default 512) or EuRoC frames (default 256) per step per GPU")
    ap.add_argument("--distinct", type=int, default=None,
                    help="synthetic base pairs / frames generated per rank (stereo default: one "
                         "per batch slot, 512 independent scenes; fewer: the batch slots are "
                         "row-rolled copies of them, all distinct; other workloads default 32)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU-baseline sample budget (0 disables)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--host-io", action="store_true",
                    help="stereo: time the PCIe-inclusive path (H2D of both views from pinned host "
                         "memory, extraction + stereo, D2H of keypoints, descriptors, uRight and "
                         "depth) instead of HBM-resident inputs")
    ap.add_argument("--input", default="resident", choices=["resident", "tensor"],
                    help="stereo: where the step's images sit in HBM: 'resident' = in the "
                         "pyramid's level-0 slots (orbx_batch_input_view; the H2D copy of a "
                         "frame lands there, so no device copy of the input is made), 'tensor' "
                         "= a caller [B, H, W] tensor copied into level 0 by the first kernel")
    ap.add_argument("--no-graphs", action="store_true",
                    help="--host-io: launch the compute sequence eagerly instead of replaying "
                         "a captured HIP graph")
    ap.add_argument("--overlap", default=None,
                    help="stereo: MODE[,FORK_LEVEL,LEVELS] side branch of each extraction "
                         "(orbx_extractor_set_overlap; 0 = every kernel in sequence; default: the "
                         "library's)")
    ap.add_argument("--serial-steps", type=int, default=20,
                    help="stereo: steps of the one-stream comparison pass after the timed region "
                         "(0: none)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="stereo: batches in flight on separate HIP streams (step i uses handle "
                         "and stream i %% inflight; 1: one batch at a time)")
    ap.add_argument("--workload", default="stereo",
                    choices=["stereo", "euroc", "reloc", "triangulation", "dropin", "kfdb", "tum",
                             "bf"],
                    help="stereo = the BASELINE metric (configs[1]); euroc = configs[2] (mono "
                         "extract + SearchByProjection vs the local map); reloc = configs[3] "
                         "(1 frame vs 10k keyframes, DB sharded); triangulation = configs[4] "
                         "(512 SearchForTriangulation jobs, sharded); dropin = the host-image "
                         "drop-in path one stereo frame at a time (per-frame latency); bf = "
                         "configs[3] as a pure brute-force top-2 (1000 query descriptors vs "
                         "--db-rows database rows, rows sharded, RCCL all-gather + merge)")
    ap.add_argument("--frames", type=int, default=300,
                    help="dropin: timed stereo frames per tracker (after --warmup frames, at least 20)")
    ap.add_argument("--trackers", default="1,2,4,8",
                    help="dropin: comma-separated numbers of concurrent tracking sessions K (each "
                         "its own left / right handles and threads, sharing the GPU); one result "
                         "line holds every K")
    ap.add_argument("--dropin-via", choices=["facade", "frame", "cabi"], default="frame",
                    help="dropin: the ORB_SLAM2::ORBextractor facade loop (tests/native/"
                         "facade_test), its one-call stereo Frame (orbx_glue::ExtractStereo), "
                         "or the bare C-ABI loop (tests/native/boundary_test)")
    ap.add_argument("--kfs", type=int, default=10000, help="reloc: keyframes in the database")
    ap.add_argument("--db-rows", type=int, default=10_000_000,
                    help="bf: database descriptors (10k keyframes x 1000, SURVEY §8(d) C4)")
    ap.add_argument("--bf-kernel", choices=["mfma", "valu"], default="mfma",
                    help="bf: the distance kernel of the line (k_bf_mfma, or north_star's XOR + "
                         "v_bcnt k_bf_top2); the other one is timed after it as alt_kernel")
    ap.add_argument("--jobs", type=int, default=512, help="triangulation: keyframe-pair jobs")
    ap.add_argument("--tri-gather", action="store_true",
                    help="triangulation: the database without its node-order copies (every "
                         "feature gathered by index, round 5's layout)")
    ap.add_argument("--queries", type=int, default=2000,
                    help="euroc: projected local-map MapPoints per frame")
    ap.add_argument("--insts-csv", default=None,
                    help="rocprofv3 --pmc CSV holding SQ_INSTS_VALU for the roofline's VALU issue "
                         "entry (default: the committed profiles/r06_pmc_insts_*.csv)")
    ap.add_argument("--traffic-csv", default=None,
                    help="comma-separated rocprofv3 --pmc counter CSVs (globs) holding FETCH_SIZE"
                         " and WRITE_SIZE for the roofline traffic field (default: the"
                         " committed profiles/ summaries of this workload)")
    return ap.parse_args()


# ---- the timed workloads' inputs (also built by tests/test_gpu_bench_geometry.py, which checks
# parity at exactly the sizes and geometries timed here) ----------------------------------------

def _gen_pair(seed):
    from my_orb_slam2_amd import synth
    return synth.stereo_pair(seed, W, H)


def stereo_inputs(rank: int, B: int, P: int):
    """configs[1] inputs of one rank: B host stereo pairs (left [B,H,W], right [B,H,W]) built
    from P generated base pairs (the headline: P = B, every slot its own scene); with P < B
    slot i is base pair i % P with both views rolled down by 37 * (i // P) rows (still
    rectified).  A pair costs ~40 ms on one host core, so more than 8 are generated by a
    process pool over this process's CPUs, forked only while the process has not touched the
    GPU.  Returns (Lh, Rh, base_pairs, distinct_slots)."""
    P = max(1, min(P, B))
    seeds = [1000 * rank + i for i in range(P)]
    pairs = None
    # not under a profiler: its preloaded library would start a GPU session in every worker
    profiled = "rocprof" in os.environ.get("LD_PRELOAD", "") or any(
        k.startswith("ROCPROF") for k in os.environ)
    if P > 8 and not profiled:
        try:
            import multiprocessing as mp
            import torch
            if not torch.cuda.is_initialized():
                with mp.get_context("fork").Pool(max(1, min(cpu_quota()[0], 8))) as pool:
                    pairs = pool.map(_gen_pair, seeds, chunksize=4)
        except Exception:
            pairs = None
    if pairs is None:
        pairs = [_gen_pair(s) for s in seeds]

    def slot(i, view):
        return np.roll(pairs[i % P][view], 37 * (i // P), axis=0)
    Lh = np.stack([slot(i, 0) for i in range(B)])
    Rh = np.stack([slot(i, 1) for i in range(B)])
    n_distinct = len({(i % P, (37 * (i // P)) % H) for i in range(B)})
    return Lh, Rh, pairs, n_distinct


def euroc_frames(rank: int, B: int, P: int):
    """configs[2] frames of one rank: P generated EuRoC-size frames, slot i = frame i % P."""
    from my_orb_slam2_amd import synth
    P = max(1, min(P, B))
    frames = [synth.frame(2000 * rank + 7 + i, EUROC_W, EUROC_H) for i in range(P)]
    return frames, [i % P for i in range(B)]


def euroc_local_maps(idx, nkp, ku, desc, queries: int, kp_cap: int, bounds):
    """Per distinct frame p: the 3-D local map SearchLocalPoints projects (synth.local_map_points
    built from the frame's own undistorted features: a camera pose, `queries` MapPoints with
    positions, normals and scale-invariance distances, their descriptors, the MapPoints already
    matched in the frame), and the motion-model pre-claimed feature mask (20 % of the
    features).  Returns {p: (pose, mps, descriptors, skip, claimed)} over the frames that slots
    `idx` reference (first slot of each)."""
    from my_orb_slam2_amd import synth
    K4, _ = synth.EUROC_CAM
    per = {}
    for b, p in enumerate(idx):
        if p not in per:
            n = int(nkp[b])
            pose, mps, d, skip = synth.local_map_points(p, ku[b, :n], desc[b, :n], queries, K4,
                                                        bounds, EUROC_W, EUROC_H)
            cl = np.random.default_rng(p).random(kp_cap) < 0.2
            per[p] = (pose, mps, d, skip, cl.astype(np.uint8))
    return per


def euroc_device_inputs(torch, dev, per, idx):
    """The EuRoC step's resident inputs, slot b = distinct frame idx[b]: frame poses, the
    concatenated local maps (slot b's MapPoints at [q_off[b], q_off[b+1])), their descriptors,
    skip masks and the pre-claimed masks; the query and nToMatch buffers the projection
    fills.  Returns a dict of device tensors plus q_off (host) and max_mps."""
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
    q_off_h = np.concatenate([[0], np.cumsum([len(per[p][1]) for p in idx])]).astype(np.int32)
    n = int(q_off_h[-1])
    return {"frames": T(np.stack([per[p][0] for p in idx])),
            "mps": T(np.concatenate([per[p][1] for p in idx])),
            "desc": T(np.concatenate([per[p][2] for p in idx])),
            "skip": T(np.concatenate([per[p][3] for p in idx])),
            "claimed": T(np.concatenate([per[p][4] for p in idx])),
            "q": torch.zeros(n * 32, dtype=torch.uint8, device=dev),
            "nvis": torch.zeros(len(idx), dtype=torch.int32, device=dev),
            "q_off": torch.from_numpy(q_off_h).to(dev), "q_off_h": q_off_h,
            "max_mps": int(np.diff(q_off_h).max()) if len(idx) else 0}


def triangulation_jobs(j0: int, j1: int):
    """configs[4] jobs [j0, j1): keyframe pairs of 2000 features each over a 100-node synthetic
    vocabulary, 30 % of the features with a MapPoint; returns (kfs, flags, F12s, epipoles)."""
    from my_orb_slam2_amd import synth
    kfs, flags, F12, epi = [], [], [], []
    for j in range(j0, j1):
        k1f, k2f, F, e, _ = synth.keyframe_pair(10000 + j, n1=2000, n2=2000, nodes=100)
        rng = np.random.default_rng(j)
        kfs += [k1f, k2f]
        flags += [rng.random(k1f.n) < 0.3, rng.random(k2f.n) < 0.3]
        F12.append(F.reshape(9))
        epi.append(e)
    return kfs, flags, F12, epi


def algorithmic_bytes_fast(level_sizes, cells_area_read, ncand):
    """k_fast: every cell ROI byte read once + one count and 4 B per candidate written."""
    return cells_area_read + 4 * ncand


_RESULT_OUT = None


def emit(line: str) -> None:
    """The one JSON result line, on the process's original stdout."""
    out = _RESULT_OUT or sys.stdout
    out.write(line + "\n")
    out.flush()


def keep_stdout_for_result() -> None:
    """Native libraries print to fd 1 (RCCL's version banner at communicator init): send fd 1
    to stderr for the rest of the run and keep a handle on the original stdout, so that the
    only thing on stdout is the result line."""
    global _RESULT_OUT
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def relaunch_if_needed(args) -> None:
    """`--gpus N` must agree with the launcher's world size.  Run without a launcher
    (no WORLD_SIZE) and N > 1, start torchrun with N ranks as a child process (nothing has
    touched the GPU yet) and exit with its status; any other mismatch is an error."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus == world:
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        import subprocess
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
               f"--master-port={29500 + os.getpid() % 1000}",
               os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    sys.exit(f"bench.py: --gpus {args.gpus} does not match WORLD_SIZE={world}")


def main():
    args = parse()
    if args.distinct is None:   # the headline: every slot its own scene
        args.distinct = (args.batch or 512) if args.workload == "stereo" else 32
    relaunch_if_needed(args)
    keep_stdout_for_result()
    if args.traffic_csv is None:
        args.traffic_csv = DEFAULT_PMC_BY_WORKLOAD.get(args.workload, DEFAULT_PMC_EUROC)
    if args.insts_csv is None:
        args.insts_csv = DEFAULT_INSTS if args.workload == "stereo" else DEFAULT_INSTS_EUROC
    if args.workload == "euroc":
        return main_euroc(args)
    if args.workload == "dropin":
        return main_dropin(args)
    if args.workload == "kfdb":
        return main_kfdb(args)
    if args.workload == "tum":
        return main_tum(args)
    if args.workload == "bf":
        return main_bf(args)
    if args.workload != "stereo":
        return main_match(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    B = args.batch or 512
    P = max(1, min(args.distinct, B))
    # every slot of the batch holds a different pair (stereo_inputs); generated before the
    # process touches the GPU (the generator pool forks)
    Lh, Rh, pairs, n_distinct = stereo_inputs(rank, B, P)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # ORBX_FORCE_DIST=1 takes the process-group path at world size 1 (torchrun
    # --nproc-per-node 1), so the RCCL timing path can be exercised on a one-GPU box
    dist_on = world > 1 or (os.environ.get("ORBX_FORCE_DIST") == "1" and "RANK" in os.environ)
    if dist_on:   # bound to this rank's GPU, so RCCL's barrier never guesses the device
        dist.init_process_group("nccl", init_method="env://", device_id=dev)

    import my_orb_slam2_amd as orbx

    Ls = torch.from_numpy(Lh).to(dev)
    Rs = torch.from_numpy(Rh).to(dev)
    torch.cuda.synchronize(dev)

    mb = float(np.float32(MBF) / np.float32(FX))
    NI = max(1, args.inflight)
    resident = args.input == "resident" and not args.host_io
    sbs, sts, run_on, run_step, overlap = headline_handles(
        torch, orbx, dev, local, B, Ls, Rs, NI, args.overlap, resident, mb)
    sb = sbs[0]

    io = None
    if args.host_io:
        # PCIe-inclusive form (never the headline): inputs start in pinned host memory and every
        # output the reference's Frame holds (mvKeys, mDescriptors, mvuRight, mvDepth) ends
        # there, double-buffered over two handles so that the H2D of batch i+1 and the D2H of
        # batch i-1 run on their own streams while batch i computes
        run_step, io, sb = host_io_pipeline(torch, orbx, dev, local, B, Lh, Rh, mb,
                                            graphs=not args.no_graphs)
        args.no_kernel_timing = True   # per-kernel events would span the overlapped copies
        sbs = [sb]

    for i in range(args.warmup):
        run_step(i)
    torch.cuda.synchronize(dev)
    if not args.no_kernel_timing:
        for h in sbs:
            h.profile(True)
            h.collect_profile()

    if dist_on:
        dist.barrier(device_ids=[local])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        run_step(i)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier(device_ids=[local])
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    prof = {}
    if not args.no_kernel_timing:
        for h in sbs:
            for k, (ms, n) in h.collect_profile().items():
                t0_, n0_ = prof.get(k, (0.0, 0))
                prof[k] = (t0_ + ms, n0_ + n)

    # sanity on the produced work (outside the timed region)
    nv = sb.nvalid.cpu().numpy()
    nkp, _, _ = sb.fetch("left")
    # every in-flight handle's outputs of its last timed step, per slot (outside the timed
    # region), for the comparison with the one-stream pass below
    dig_inflight = [stereo_digests(h) for h in sbs] if io is None else None

    # The same step with every kernel in sequence on one stream and one batch in flight
    # (outside the timed region): the overlap's gain measured in this run, and each kernel's
    # launch time on its own (in the timed run the side branch and the other batch in flight
    # share the device with every launch, so the HIP-event spans include that sharing)
    serial = dig_serial = None
    if args.serial_steps > 0 and io is None:
        for h in sbs:
            h.ext.set_overlap(0)
        for i in range(3):
            run_on(sbs[0], sts[0])
        torch.cuda.synchronize(dev)
        if not args.no_kernel_timing:
            for h in sbs:   # the warm-up steps' launches are not part of the pass
                h.collect_profile()
        ts = time.perf_counter()
        for i in range(args.serial_steps):
            run_on(sbs[0], sts[0])
        torch.cuda.synchronize(dev)
        t_ser = time.perf_counter() - ts
        serial = {"steps": args.serial_steps, "ms_per_step": 1000.0 * t_ser / args.serial_steps,
                  "value": B * args.serial_steps / t_ser}
        dig_serial = stereo_digests(sbs[0])
        if not args.no_kernel_timing:
            sprof = {}
            for h in sbs:
                for k, (ms, n) in h.collect_profile().items():
                    t0_, n0_ = sprof.get(k, (0.0, 0))
                    sprof[k] = (t0_ + ms, n0_ + n)
            serial["kernel_ms_per_step"] = {k: round(v[0] / args.serial_steps, 4)
                                            for k, v in sprof.items()}
            serial["prof"] = sprof
        for h in sbs:
            h.ext.set_overlap(*overlap)

    verify = verification(dig_inflight, dig_serial, B)

    total_pairs = B * args.steps * world
    fps = total_pairs / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # roofline of the dominant kernel: the largest kernel group of the one-stream pass (the
    # run's own measurement of each kernel alone), its launches timed in the timed region
    roof = None
    if prof:
        sprof = serial.get("prof") if serial else None
        roof = headline_roofline(prof, args.steps, sprof, args.serial_steps, sb.ext, B,
                                 args.traffic_csv, args.insts_csv)
        roof["overlap"] = {"mode": overlap[0], "fork_level": overlap[1], "levels": overlap[2]}
        add_valu_floor(roof, ms_per_step)
    if serial:
        serial.pop("prof", None)
        serial.pop("kernel_ms_per_step", None)

    cpu = cpu_tp = cpu_tp_all = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        ref = dig_serial or (dig_inflight[0] if dig_inflight else None)
        cpu = cpu_baseline(pairs, mb, args.cpu_seconds,
                           gpu_digests=ref[:min(P, 8)] if ref else None)
        # SURVEY §8(d) mode (ii): one worker per CPU this process may use (the cgroup's share),
        # and one per host CPU (os.cpu_count(); above the share the workers only time-slice)
        cpu_tp = cpu_baseline_throughput(pairs, mb, min(args.cpu_seconds, 6.0),
                                         workers=cpu_quota()[0])
        cpu_tp_all = cpu_baseline_throughput(pairs, mb, min(args.cpu_seconds, 6.0))

    if rank == 0:
        out = {"metric": METRIC, "value": fps, "unit": "frames/sec", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "u8", "data": "synthetic",
               "config": {"workload": "kitti_stereo_extract_match", "width": W, "height": H,
                          "nfeatures": NFEAT, "nlevels": 8, "scale_factor": 1.2,
                          "pairs_per_step_per_gpu": B, "distinct_pairs": n_distinct,
                          "base_pairs": P, "inflight_batches": NI,
                          "parallelism": f"dp{world}"},
               "mean_keypoints_left": float(nkp.mean()),
               "mean_stereo_matches": float(nv.mean()),
               "verified": verify["verified"] if verify else None, "verification": verify,
               "roofline": roof, "cpu_baseline": cpu, "cpu_baseline_throughput": cpu_tp,
               "cpu_baseline_throughput_all_host_cpus": cpu_tp_all, "one_stream": serial}
        if io is not None:
            out["metric"] = METRIC + " (PCIe-inclusive: host images in, host keypoints out)"
            out["config"]["host_io"] = io
            out["pcie_bound_frac"] = fps / io["pcie_bound_pairs_per_s"]
        emit(json.dumps(out))
    if dist_on:
        dist.destroy_process_group()


def headline_handles(torch, orbx, dev, local, B, Ls, Rs, NI, overlap_arg, resident, mb):
    """The timed configuration of the headline: NI StereoBatch handles of B pairs, step i on
    handle i % NI and stream i % NI (stream 0 = the current stream), every extraction with the
    side branch `overlap_arg` ("MODE,FORK,LEVELS"; None = the library's default); with
    `resident` the B pairs sit in each handle's level-0 slots (written once, here), else they
    are copied in from the Ls / Rs tensors by the first kernel.  tests/test_gpu_bench_geometry.py
    runs exactly this.  Returns (handles, raw streams, run_on(handle, stream), run_step(i),
    overlap tuple)."""
    sbs = [orbx.StereoBatch(B, NFEAT, 1.2, 8, 20, 7, device=local) for _ in range(NI)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(NI - 1)]
    sts = [s_.cuda_stream for s_ in streams]
    if overlap_arg is not None:
        ov = [int(v) for v in str(overlap_arg).split(",")]
        for h in sbs:
            h.ext.set_overlap(*ov)
    overlap = sbs[0].ext.overlap()
    if resident:
        for h in sbs:
            Lv, Rv = h.input_views(W, H)
            Lv.copy_(Ls)
            Rv.copy_(Rs)
        torch.cuda.synchronize(dev)

        def run_on(h, st):
            h.run_resident(MBF, mb, stream=st)
    else:
        def run_on(h, st):
            h(Ls, Rs, MBF, mb, stream=st)

    def run_step(i):
        run_on(sbs[i % NI], sts[i % NI])
    return sbs, sts, run_on, run_step, overlap


def slot_digest(kl, dl, kr, dr, u, z, nv) -> str:
    """SHA-256 of one stereo frame's outputs: left / right keypoints (cv::KeyPoint records) and
    descriptors, uRight and depth of the left keypoints, and the valid-match count."""
    import hashlib
    h = hashlib.sha256()
    for a in (kl, dl, kr, dr, u, z):
        a = np.zeros(0, np.uint8) if a is None else np.ascontiguousarray(a)
        h.update(int(a.shape[0]).to_bytes(8, "little"))
        h.update(a.tobytes())
    h.update(int(nv).to_bytes(8, "little", signed=True))
    return h.hexdigest()


def stereo_digests(sb) -> list:
    """slot_digest of every pair of a StereoBatch's last call (host copies of its outputs)."""
    nkl, kl, dl = sb.fetch("left")
    nkr, kr, dr = sb.fetch("right")
    B = len(nkl)
    u = sb.uR[:B].cpu().numpy()
    z = sb.depth[:B].cpu().numpy()
    nv = sb.nvalid[:B].cpu().numpy()
    return [slot_digest(kl[i, :nkl[i]], dl[i, :nkl[i]], kr[i, :nkr[i]], dr[i, :nkr[i]],
                        u[i, :nkl[i]], z[i, :nkl[i]], nv[i]) for i in range(B)]


def verification(dig_inflight, dig_serial, B):
    """`verified`: every in-flight handle's last timed step equals the one-stream pass of the
    same pairs, slot by slot (or, without that pass, the in-flight handles equal each other)."""
    if not dig_inflight:
        return None
    import hashlib
    ref = dig_serial if dig_serial is not None else dig_inflight[0]
    bad = [(k, i) for k, d in enumerate(dig_inflight) for i in range(B) if d[i] != ref[i]]
    return {"verified": not bad, "slots": B, "handles": len(dig_inflight),
            "against": "one-stream pass (overlap 0, one batch in flight)" if dig_serial is not None
                       else "the first in-flight handle",
            "mismatched_slots": len(bad), "first_mismatches": bad[:8],
            "digest": hashlib.sha256("".join(ref).encode()).hexdigest()[:16]}


def host_io_pipeline(torch, orbx, dev, local, B, Lh, Rh, mb, graphs=True):
    """The PCIe-inclusive stereo step, pipelined: two StereoBatch handles alternate batches;
    per batch one H2D copy (a 2-D copy whose rows are whole images, pinned host memory laid
    out with the pyramid's row pitch) lands the 2B views straight in the handle's level-0
    slots, the extraction + stereo run on the handle's stream (replayed from a HIP graph of the
    launch sequence when `graphs`), and four D2H copies return keypoints, descriptors, uRight
    and depth to pinned host buffers.  H2D and D2H have a stream each; events order a handle's
    next H2D after its previous compute and its next compute after its previous D2H.  Returns
    (run_step, io description, the first handle)."""
    import ctypes
    from my_orb_slam2_amd._lib import check
    hip = ctypes.CDLL("libamdhip64.so")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    hip.hipMemcpy2DAsync.argtypes = [vp, sz, vp, sz, sz, sz, ctypes.c_int, vp]
    hs = [orbx.StereoBatch(B, NFEAT, 1.2, 8, 20, 7, device=local) for _ in range(2)]
    # one stream per handle: the link is the bound here, and the side branches' two extra
    # streams would share the device's 4 hardware queues with the copy streams (88 % of the
    # PCIe bound with them, 98-103 % without)
    for h in hs:
        h.ext.set_overlap(0)
    base, pitch, istride = [], None, None
    for h in hs:
        h.input_views(W, H)          # prepares the workspace and the output tensors
        p_, pi_, st_ = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_size_t()
        check("orbx_batch_input_view", h.ext._L.orbx_batch_input_view(
            h.ext._h, W, H, 2 * B, ctypes.byref(p_), ctypes.byref(pi_), ctypes.byref(st_)))
        base.append(p_.value)
        pitch, istride = pi_.value, st_.value
    src = torch.zeros((2 * B, H, pitch), dtype=torch.uint8).pin_memory()
    src[:B, :, :W] = torch.from_numpy(Lh)
    src[B:, :, :W] = torch.from_numpy(Rh)
    s_h2d, s_d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    s_comp = [torch.cuda.Stream(dev) for _ in range(2)]
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_comp = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]

    def h2d(k, stream):
        if hip.hipMemcpy2DAsync(base[k], istride, src.data_ptr(), H * pitch, H * pitch, 2 * B,
                                1, vp(stream.cuda_stream)) != 0:
            raise RuntimeError("hipMemcpy2DAsync H2D failed")

    def d2h(k, stream):
        vv = hs[k].ext.batch_view()
        for dst, srcp, n in ((outs[k][0], vv.kps, kpb), (outs[k][1], vv.desc, dsb),
                             (outs[k][2], hs[k].uR.data_ptr(), fb),
                             (outs[k][3], hs[k].depth.data_ptr(), fb)):
            if hip.hipMemcpyAsync(dst.data_ptr(), srcp, n, 2, vp(stream.cuda_stream)) != 0:
                raise RuntimeError("hipMemcpyAsync D2H failed")

    for k in range(2):   # one eager run per handle: workspace warm, batch view published
        h2d(k, s_comp[k])
        hs[k].run_resident(MBF, mb, stream=s_comp[k].cuda_stream)
        s_comp[k].synchronize()
    kc = hs[0].ext.batch_view().kp_cap
    kpb, dsb, fb = 2 * B * kc * 28, 2 * B * kc * 32, B * kc * 4
    outs = [[torch.empty(n, dtype=torch.uint8).pin_memory() for n in (kpb, dsb, fb, fb)]
            for _ in range(2)]
    gr = [None, None]
    for k in range(2):   # then the graph capture of the same launch sequence
        if graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s_comp[k]):
                hs[k].run_resident(MBF, mb, stream=s_comp[k].cuda_stream)
            gr[k] = g
    torch.cuda.synchronize(dev)

    def run_step(i):
        k = i % 2
        s_h2d.wait_event(ev_comp[k])           # the handle's last batch has left level 0
        h2d(k, s_h2d)
        ev_in[k].record(s_h2d)
        s_comp[k].wait_event(ev_in[k])
        s_comp[k].wait_event(ev_out[k])        # its last outputs have reached the host
        if gr[k] is not None:
            with torch.cuda.stream(s_comp[k]):
                gr[k].replay()
        else:
            hs[k].run_resident(MBF, mb, stream=s_comp[k].cuda_stream)
        ev_comp[k].record(s_comp[k])
        s_d2h.wait_event(ev_comp[k])
        d2h(k, s_d2h)
        ev_out[k].record(s_d2h)

    # the PCIe bound of this step on this box: the same copies alone, each direction alone and
    # both at once (on their own streams), 10 repetitions
    def timed(fn, reps=10):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps
    t_h2d = timed(lambda: h2d(0, s_h2d))
    t_d2h = timed(lambda: d2h(0, s_d2h))
    t_both = timed(lambda: (h2d(1, s_h2d), d2h(0, s_d2h)))
    h2d_bytes, d2h_bytes = 2 * B * H * pitch, kpb + dsb + 2 * fb
    io = {"pipeline": "2 handles, H2D / compute / D2H on separate streams" +
                      (", compute replayed from HIP graphs" if graphs else ""),
          "h2d_bytes_per_step": h2d_bytes, "d2h_bytes_per_step": d2h_bytes,
          "h2d_gbs": h2d_bytes / t_h2d / 1e9, "d2h_gbs": d2h_bytes / t_d2h / 1e9,
          "copies_only_ms_per_step": 1000.0 * t_both,
          "pcie_bound_pairs_per_s": B / t_both}
    return run_step, io, hs[0]


# kernel groups of the stereo step: the pyramid's two kinds of launch apart (level 0 blurs the
# input slot, levels 1-7 resize + blur), then the other kernels
HEADLINE_GROUPS = ("k_level0", "k_level1_7", "k_fast", "k_octree", "k_orient_desc", "k_stereo")
# launches per step of each group in the one-stream step (overlap 0, one batch in flight): the
# launch count of the PMC passes (tools/prof_counters.sh), whose per-dispatch averages scale by it
ONE_STREAM_LAUNCHES = {"k_level": 8, "k_level0": 1, "k_level1_7": 7, "k_fast": 1, "k_octree": 1,
                       "k_orient_desc": 1, "k_stereo": 1}


def split_level(prof):
    """{group: (total_ms, launches)} with k_level split into k_level0 and k_level1_7 (the
    library times level 0's launches under both k_level and k_level0)."""
    out = {k: v for k, v in prof.items() if v[1]}
    if "k_level" in out:
        t_all, n_all = out["k_level"]
        t0, n0 = out.get("k_level0", (0.0, 0))
        if n_all - n0 > 0:
            out["k_level1_7"] = (t_all - t0, n_all - n0)
    return out


def step_bytes(ext, n, B):
    """Algorithmic HBM bytes per STEP of each kernel group (kernel_bytes per one-stream launch x
    the one-stream launches per step)."""
    return {k: v * ONE_STREAM_LAUNCHES.get(k, 1) for k, v in kernel_bytes(ext, n, B).items()}


def traffic_per_step(paths, kernel):
    """PMC HBM bytes per step of a kernel group: the per-dispatch average of the one-stream PMC
    passes x that pass's launches per step."""
    t = traffic_from_csv(paths, kernel)
    return t * ONE_STREAM_LAUNCHES.get(kernel, 1) if t else t


def roofline_entry(name, tot_ms, launches, steps, alg_step, traffic_step):
    """One kernel group against the HBM roof: algorithmic bytes per launch (the step's bytes
    over its launches per step; capped by the measured traffic, counted_bytes) / the mean
    HIP-event launch duration."""
    per_step = launches / max(steps, 1)
    req = alg_step / per_step if alg_step else None
    traffic = traffic_step / per_step if traffic_step else None
    alg = counted_bytes(req, traffic)
    avg_s = tot_ms / 1000.0 / max(launches, 1)
    ach = (alg / avg_s / 1e9) if (alg and avg_s > 0) else None
    return {"kernel": name, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (ach / HBM_PEAK_GBS) if ach else None, "traffic": traffic,
            "algorithmic_bytes_per_launch": alg, "requested_bytes_per_launch": req,
            "avg_launch_ms": avg_s * 1000.0, "launches_per_step": per_step,
            "ms_per_step": tot_ms / max(steps, 1)}


def pick_dominant(gprof, steps):
    """The kernel group with the most time per step (one stream: kernels do not overlap)."""
    cand = {k: v for k, v in gprof.items() if k in HEADLINE_GROUPS}
    return max(cand, key=lambda k: cand[k][0] / max(steps, 1)) if cand else None


def headline_roofline(prof, steps, sprof, ssteps, ext, B, traffic_csv, insts_csv, ta_csv=None):
    """The headline `roofline` object.  `kernel` is the group that takes the most time in the
    run's one-stream pass (`sprof` over `ssteps` steps; the timed profile when the run has no
    such pass); `frac` is that group's algorithmic bytes per launch over its mean launch
    duration in the timed region (hipExtLaunchKernel events from the kernel's own dispatch,
    the quantity rocprofv3 --kernel-trace reports).  `serial_pass` is the same group timed in
    the one-stream pass; `per_kernel` holds every group, from the one-stream pass."""
    gt = split_level(prof)
    gs = split_level(sprof) if sprof else None
    dom = pick_dominant(gs if gs else gt, ssteps if gs else steps)
    geo = step_bytes(ext, 2 * B, B)
    if dom is None or dom not in gt:
        return None
    roof = roofline_entry(dom, *gt[dom], steps, geo.get(dom), traffic_per_step(traffic_csv, dom))
    roof["selected_by"] = ("largest kernel group per step in the one-stream pass" if gs else
                           "largest kernel group per step in the timed region")
    roof["kernel_ms_per_step"] = {k: round(v[0] / max(steps, 1), 4) for k, v in gt.items()}
    kp, ks = (gs, ssteps) if gs else (gt, steps)
    roof["per_kernel_source"] = "one-stream pass (one_stream)" if gs else "timed region"
    roof["per_kernel"] = {k: roofline_entry(k, *kp[k], ks, geo.get(k),
                                            traffic_per_step(traffic_csv, k))
                          for k in HEADLINE_GROUPS + ("k_level",) if k in kp}
    roof["one_stream_ms_per_step"] = {k: round(v[0] / max(ks, 1), 4) for k, v in kp.items()}
    # the integer kernels are bound by VALU issue, not HBM: the same launches against the
    # issue rate (SQ_INSTS_VALU from a PMC pass of the same workload)
    # (the PMC pass counts one-stream dispatches: scaled to this entry's launches per step)
    for e in [roof] + list(roof["per_kernel"].values()):
        e["valu"] = valu_entry(insts_csv, e["kernel"], e["avg_launch_ms"] / 1000.0,
                               ONE_STREAM_LAUNCHES.get(e["kernel"], 1) / e["launches_per_step"])
    if gs and dom in gs:
        se = roof["per_kernel"][dom]
        roof["serial_pass"] = {"avg_launch_ms": se["avg_launch_ms"], "achieved": se["achieved"],
                               "frac": se["frac"], "launches_per_step": se["launches_per_step"]}
    # the kernel group that takes the most time per step in the timed (scheduled) region, the
    # one a rocprofv3 summary of this command ranks first
    tdom = max((k for k in gt if k in HEADLINE_GROUPS), key=lambda k: gt[k][0], default=None)
    if tdom:
        tot = sum(v[0] for v in gt.values())
        roof["timed_dominant"] = {"kernel": tdom, "ms_per_step": round(gt[tdom][0] / max(steps, 1), 4),
                                  "share_of_kernel_time": round(gt[tdom][0] / tot, 4) if tot else None,
                                  "hbm_frac": roofline_entry(tdom, *gt[tdom], steps, geo.get(tdom),
                                                             traffic_per_step(traffic_csv, tdom))["frac"]}
    for e in [roof] + list(roof["per_kernel"].values()):
        label_binding_roof(e)
        # the texture addresser's busy fraction (the unit a patch-staging kernel can saturate
        # below its VALU and HBM roofs: k_orient_desc), from the one-stream TA pass
        t = ta_busy_from_csv(DEFAULT_TA if ta_csv is None else ta_csv, e["kernel"])
        if t is not None:
            e["ta_busy"] = t
    return roof


DEFAULT_TA = os.path.join(HERE, "profiles", "r06_pmc_ta_b512.csv")


def ta_busy_from_csv(paths, kernel):
    """TA_BUSY_avr (cycles per texture addresser, averaged over the TAs) over the launch's
    GRBM_GUI_ACTIVE / 8 cycles (GRBM counts over the 8 XCDs) from a rocprofv3 TA pass, per
    dispatch, or None when the pass does not hold the kernel."""
    busy = counter_from_csv(paths, kernel, "TA_BUSY_avr")
    grbm = counter_from_csv(paths, kernel, "GRBM_GUI_ACTIVE")
    return busy / (grbm / 8.0) if busy and grbm else None


VALU_ISSUE_PEAK = 1024 * 2.4e9 / 1e12   # T SIMD issue cycles/s (1024 SIMDs at 2.4 GHz)


def valu_floor_ms(per_kernel):
    """The step's VALU issue floor: every kernel group's wave instructions per step (PMC
    SQ_INSTS_VALU per launch x launches per step) x its mean issue cycles per instruction (the
    opcode mix priced at the measured gfx950 rates), over 1024 SIMDs x 2.4 GHz.  None if any
    group lacks a VALU entry."""
    cyc = 0.0
    for k in HEADLINE_GROUPS:
        e = per_kernel.get(k)
        v = (e or {}).get("valu") or {}
        if e is None:
            continue
        if not v.get("wave_instr_per_launch") or not v.get("mean_issue_cycles"):
            return None
        cyc += v["wave_instr_per_launch"] * e["launches_per_step"] * v["mean_issue_cycles"]
    return 1000.0 * cyc / (VALU_ISSUE_PEAK * 1e12)


def add_valu_floor(roof, ms_per_step):
    """roof["valu_floor_ms"] (valu_floor_ms over the one-stream per_kernel entries) and
    roof["valu_floor_frac"] = that floor over the timed step: how close the step is to the
    roof that binds the integer pipeline chip-wide."""
    f = valu_floor_ms(roof.get("per_kernel") or {})
    roof["valu_floor_ms"] = f
    roof["valu_floor_frac"] = f / ms_per_step if f and ms_per_step > 0 else None


def label_binding_roof(e):
    """Name the roof the counters show for a roofline entry: the larger of its VALU issue
    fraction (the mix-aware busy fraction from the PMC passes) and its HBM fraction.  When VALU
    is larger, `bound` is "valu" and achieved / peak / frac are VALU issue cycles per second
    against 1024 SIMDs x 2.4 GHz; the HBM figures move to `hbm` either way.  `traffic` stays
    the PMC HBM bytes per launch."""
    v = e.get("valu") or {}
    busy = v.get("busy_frac")
    hbm = {"achieved": e.get("achieved"), "peak": e.get("peak"), "unit": e.get("unit"),
           "frac": e.get("frac")}
    if busy is None or busy <= (e.get("frac") or 0):
        e["hbm"] = hbm
        return
    ach = v["wave_instr_per_launch"] * v["mean_issue_cycles"] / (e["avg_launch_ms"] / 1000.0) / 1e12
    e.update({"bound": "valu", "achieved": ach, "peak": VALU_ISSUE_PEAK,
              "unit": "T VALU issue cycles/s", "frac": ach / VALU_ISSUE_PEAK, "hbm": hbm})


def counted_bytes(requested, traffic):
    """Bytes a roofline entry credits to one launch: the kernel's requested (algorithmic)
    bytes, capped by the measured HBM traffic when a PMC pass holds it.  Requested bytes
    count overlapping reads in full (k_orient_desc: every keypoint's 31x31 and 37x37
    patches), which the caches serve once, so uncapped they would overstate the HBM
    fraction."""
    if not requested:
        return requested
    return min(requested, traffic) if traffic else requested


def kernel_bytes(ext, n, B):
    """Algorithmic HBM bytes per launch of each kernel.  One
    launch covers the n images (k_level: one level of them); B stereo pairs for k_stereo."""
    v = ext.batch_view()
    L = 8
    area = [v.level_w[l] * v.level_h[l] for l in range(L)]
    kc = v.kp_cap
    return {
        # §8(d): the input is read once and never copied; level l >= 1 reads level l-1 and
        # writes itself and its blur, level 0 reads the input and writes its blur (a device
        # copy of the input, made only when the caller's images are not in the level-0 slots,
        # is not algorithmic work): (sum_{l<L-1} A_l + 2 sum A) per step, averaged per launch
        "k_level": n * (sum(area[:-1]) + 2 * sum(area)) / L,
        "k_level0": n * 2 * area[0],
        "k_level1_7": n * (sum(area[:-1]) + 2 * sum(area[1:])) / (L - 1),
        # every level byte read once
        "k_fast": n * sum(area),
        # candidates in (<= 4 B each, bounded by 2 x kp slots here) and survivors out
        "k_octree": n * 4 * kc * 2,
        # 31x31 raw + 37x37 blurred patch in, 28 + 32 B out per keypoint
        "k_orient_desc": n * kc * (31 * 31 + 37 * 37 + 60),
        # both views' keypoints + descriptors in, 11x11 + 11x21 SAD windows, 8 B out
        "k_stereo": B * kc * (2 * (28 + 32) + 11 * 11 + 11 * 21 + 8),
    }


# bench names of kernel groups -> the kernel-name pattern of their dispatches in rocprofv3 CSVs
CSV_NAME = {"k_level0": "k_level_strip<4>", "k_level1_7": "k_level_strip<3>"}


def counter_from_csv(paths, kernel, counter):
    """Counter value per dispatch of `kernel` (summed over a dispatch's rows), averaged over
    its dispatches in rocprofv3 --pmc CSVs, or None."""
    import csv
    import glob
    pat = CSV_NAME.get(kernel, kernel)
    tot, ids = 0.0, set()
    for p in (paths or "").split(","):
        for path in (sorted(glob.glob(p.strip())) if p.strip() else []):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if pat in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                        tot += float(row["Counter_Value"])
                        ids.add((path, row.get("Dispatch_Id")))
    return tot / len(ids) if ids else None


def valu_from_csv(paths, kernel):
    return counter_from_csv(paths, kernel, "SQ_INSTS_VALU")


ISA_MIX = os.path.join(HERE, "profiles", "r06_isa_mix.json")


def _mangled_key(demangled: str) -> str:
    """'void orbx::k_level_strip<3>(...)' -> 'k_level_stripILi3E' (the form of the kernel's
    symbol in tools/isa_mix.py's table); 'void orbx::k_fast(...)' -> '6k_fastE'."""
    import re
    m = re.search(r"(k_\w+)(<(-?\d+)>)?\(", demangled)
    if not m:
        return ""
    name, targ = m.group(1), m.group(3)
    return f"{name}ILi{targ}E" if targ is not None else f"{len(name)}{name}E"


def mix_cycles_from_csv(paths, kernel, mix_path=None):
    """Mean issue cycles per VALU instruction of a kernel group: each dispatch's SQ_INSTS_VALU
    weighted by its kernel's static opcode-mix cost (tools/isa_mix.py, profiles/r05_isa_mix.json)."""
    import csv
    import glob
    try:
        mix = json.load(open(mix_path or ISA_MIX))
    except OSError:
        return None
    pat = CSV_NAME.get(kernel, kernel)
    num = den = 0.0
    for p in (paths or "").split(","):
        for path in (sorted(glob.glob(p.strip())) if p.strip() else []):
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = row.get("Kernel_Name", "")
                    if pat not in name or row.get("Counter_Name") != "SQ_INSTS_VALU":
                        continue
                    key = _mangled_key(name)
                    costs = [v["mean_cycles"] for k, v in mix.items() if key and key in k
                             and v.get("mean_cycles")]
                    if not costs:
                        continue
                    num += float(row["Counter_Value"]) * costs[0]
                    den += float(row["Counter_Value"])
    return num / den if den else None


def valu_entry(paths, kernel, avg_s, scale=1.0):
    """A launch against the VALU issue roof:
    * busy_frac (mix-aware, <= 1 at the nominal clock): SQ_INSTS_VALU x the kernel's mean
      issue cycles per VALU instruction (its opcode mix priced at the measured gfx950 rates,
      tools/isa_mix.py) over the SIMDs' cycles of the launch (1024 SIMDs x the HIP-event launch
      time x 2.4 GHz; the clock drops under load, so this is a lower bound);
    * valubusy_4cycle: rocprof's VALUBusy (SQ_ACTIVE_INST_VALU, 4 cycles per instruction
      whatever its rate, over GRBM_GUI_ACTIVE / 8 cycles: overstates full-rate-rich kernels,
      may exceed 1, and the GRBM cycles of launches under ~0.3 ms read high), for reference;
    * the issue rate in wave instructions/s (SQ_INSTS_VALU over the HIP-event launch time).
    `scale` converts the PMC pass's per-dispatch count to one launch of the entry (a kernel the
    timed schedule launches twice per step where the one-stream pass launches it once: 1/2)."""
    v = valu_from_csv(paths, kernel)
    if v:
        v *= scale
    act = counter_from_csv(paths, kernel, "SQ_ACTIVE_INST_VALU")
    grbm = counter_from_csv(paths, kernel, "GRBM_GUI_ACTIVE")
    if not v and not act:
        return None
    out = {"bound": "valu"}
    cyc = mix_cycles_from_csv(paths, kernel)
    if v and cyc and avg_s > 0:
        cycles = avg_s * 2.4e9
        out.update({"busy_frac": v * cyc / (1024.0 * cycles), "mean_issue_cycles": cyc,
                    "cycles": cycles})
    if act and grbm:
        out["valubusy_4cycle"] = 4.0 * act / (1024.0 * grbm / 8.0)
    if v and avg_s > 0:
        out.update({"wave_instr_per_launch": v, "issue_rate": v / avg_s / 1e12,
                    "unit": "T wave-instr/s"})
    return out


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
    pat = CSV_NAME.get(kernel, kernel)
    per = {}
    for path in files:
        with open(path) as f:
            for row in csv.DictReader(f):
                if pat not in row.get("Kernel_Name", ""):
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


def cpu_model() -> str:
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return model


def latency_stats(ms) -> dict:
    """Median / mean of per-frame latencies, as Examples/Stereo/stereo_kitti.cc:115-123 prints
    them (sorted vector, element n/2; plain mean)."""
    v = sorted(ms)
    return {"median_ms": v[len(v) // 2], "mean_ms": sum(v) / len(v), "p90_ms": v[int(0.9 * len(v))],
            "frames": len(v)}


def cpu_baseline(pairs, mb, budget_s, min_frames=200, warmup=20, gpu_digests=None):
    """The CPU restatement timed on this host in the reference's own mode (src/Frame.cc:89-102:
    left and right extraction on two threads, then ComputeStereoMatches on one), per stereo
    frame: `warmup` untimed frames, then at least `min_frames` timed ones (more while the
    budget lasts); median and mean latency like stereo_kitti.cc:115-123, value = frames/s over
    the timed frames.  The first warm-up frames are the base pairs, i.e. batch slots 0..P-1:
    their outputs are checked against the GPU's (`gpu_digests`, bench.slot_digest of those
    slots) before the timed frames start."""
    try:
        import oracle
    except Exception:
        return None
    ol = oracle.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
    orr = oracle.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
    ms = []
    t_start = None
    f = 0
    checked, agree = 0, 0
    ncheck = min(len(gpu_digests or []), warmup, len(pairs))
    while True:
        Lp, Rp = pairs[f % len(pairs)]
        t0 = time.perf_counter()
        res = {}
        th = threading.Thread(target=lambda: res.__setitem__("r", orr(Rp)))
        th.start()
        kl, dl = ol(Lp)
        th.join()
        u, z, nv = oracle.stereo_match(ol, orr, len(kl), MBF, mb)
        t1 = time.perf_counter()
        if f < ncheck:      # a warm-up frame: outside the timed frames
            kr, dr = res["r"]
            checked += 1
            agree += slot_digest(kl, dl, kr, dr, u, z, nv) == gpu_digests[f]
        f += 1
        if f == warmup:
            t_start = time.perf_counter()
        elif f > warmup:
            ms.append(1000.0 * (t1 - t0))
            if len(ms) >= min_frames and t1 - t_start >= budget_s:
                break
    el = time.perf_counter() - t_start
    out = {"value": len(ms) / el, "unit": "frames/sec", "cores": 2, "kind": "port",
           "sample": f"{len(ms)} KITTI-size synthetic stereo pairs after {warmup} warm-up pairs, "
                     f"L/R extraction on 2 threads + ComputeStereoMatches (Frame.cc:89-102), "
                     f"{el:.1f} s",
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
           "build": f"g++ -O3 -march={oracle.ISA} -ffp-contract=off (oracle/Makefile)"}
    if ncheck:
        out["gpu_slots_checked"] = checked
        out["gpu_slots_equal"] = agree
    out.update(latency_stats(ms))
    return out


def cpu_quota():
    """(CPUs this process may run on: the affinity set capped by the cgroup CPU quota, the
    quota as text or None).  On the GPU box os.cpu_count() shows the whole machine (256) while
    the cgroup grants the GPU's share."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(path).read().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and txt and txt[0] != "max":
            q = f"{txt[0]}/{txt[1]}"
            n = min(n, max(1, -(-int(txt[0]) // int(txt[1]))))
        elif path.endswith("cfs_quota_us") and txt and int(txt[0]) > 0:
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            q = f"{txt[0]}/{per}"
            n = min(n, max(1, -(-int(txt[0]) // per)))
        break
    return n, q


def cpu_baseline_throughput(pairs, mb, budget_s, workers=None):
    """SURVEY §8(d) mode (ii): one stereo-frame pipeline per core (extract L, extract R,
    ComputeStereoMatches, each worker with its own extractors) on every host CPU by default
    (`workers` = os.cpu_count(); ctypes releases the GIL inside the restatement).  Reports the
    aggregate frames/s and the per-pair median / mean latency of the workers' frames."""
    try:
        import oracle
    except Exception:
        return None
    usable, quota = cpu_quota()
    workers = workers or os.cpu_count() or 1
    lat = [[] for _ in range(workers)]
    stop = [False]
    go = threading.Barrier(workers + 1)

    def work(w):
        ol = oracle.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
        orr = oracle.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
        i = w
        go.wait()
        while not stop[0]:
            Lp, Rp = pairs[i % len(pairs)]
            t0 = time.perf_counter()
            kl, _ = ol(Lp)
            orr(Rp)
            oracle.stereo_match(ol, orr, len(kl), MBF, mb)
            lat[w].append(1000.0 * (time.perf_counter() - t0))
            i += workers
    ths = [threading.Thread(target=work, args=(w,)) for w in range(workers)]
    for t in ths:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    time.sleep(budget_s)
    stop[0] = True
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    allms = [v for l_ in lat for v in l_]
    out = {"value": len(allms) / el, "unit": "frames/sec", "cores": workers, "kind": "port",
           "sample": f"{len(allms)} KITTI-size synthetic stereo pairs on {workers} worker threads "
                     f"(one pipeline per core, SURVEY §8d mode ii), {el:.1f} s",
           "host_cpus": os.cpu_count(), "usable_cpus": usable, "cgroup_cpu_quota": quota}
    if allms:
        out.update(latency_stats(allms))
    return out


# ---- the drop-in host path, one stereo frame at a time ---------------------------------------

def main_dropin(args):
    """The path INTEGRATION.md installs into ORB-SLAM2, timed as its Tracking thread runs it:
    per stereo frame a Frame through the compiled facade (tests/native/facade_test.cpp
    `bench`), host memory in and out (PCIe included), so no Python overhead enters the
    latency.  --dropin-via frame (the default): the stereo Frame's extraction and matching as
    one call, orbx_glue::ExtractStereo (both views as one two-image submission with the stereo
    match appended); facade: the reference's two ExtractORB threads (src/Frame.cc:89-92), then
    ComputeStereoMatches (:102); cabi: the same on the bare C ABI (boundary_test.cpp `bench`).
    `--trackers K[,K..]`: K independent sessions (System.cc:91-101 each) run that loop at once
    on their own handles and threads, sharing the GPU; per K the per-frame median / mean over
    every session's --frames frames after --warmup (>= 20) frames, and the aggregate pairs/s
    (all sessions' frames over the wall time of the timed frames).  Every session's output
    digest must agree (the same pairs in the same order).  With --dropin-via frame the
    two-thread facade loop runs too (`two_thread_facade`), and its digests must equal the
    one-call loop's.  Beside it the CPU restatement run the same way on the same pairs."""
    import subprocess
    import tempfile
    B = max(1, min(args.distinct, 32))
    Lh, Rh, pairs, _ = stereo_inputs(0, B, B)
    mb = float(np.float32(MBF) / np.float32(FX))
    warm = max(20, args.warmup)
    ks = [max(1, int(k)) for k in str(args.trackers).split(",")]

    def loop(d, via):
        binp = os.path.join(ROOT, "tests", "native",
                            "boundary_test" if via == "cabi" else "facade_test")
        extra = ["frame"] if via == "frame" else (["pyr"] if via == "pyr" else [])
        per_k, digests = {}, {}
        for K in ks:
            r = subprocess.run([binp, "bench", d, str(args.frames), str(warm), str(K)] + extra,
                               capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                sys.exit(f"bench.py: {binp} failed ({r.returncode}): {r.stderr[-2000:]}")
            res = json.loads(r.stdout.strip().splitlines()[-1])
            per_k[K] = {"trackers": K, "latency": latency_stats(res["latency_ms"]),
                        "pairs_per_s": K * args.frames / (res["wall_ms"] / 1000.0),
                        "wall_ms": res["wall_ms"],
                        "sessions_agree": len(set(res["digests"])) == 1,
                        "mean_keypoints_left": res["mean_keypoints_left"],
                        "mean_stereo_matches": res["mean_stereo_matches"]}
            digests[K] = res["digests"]
        return per_k, digests

    with tempfile.TemporaryDirectory() as d:
        for i in range(B):
            Lh[i].tofile(os.path.join(d, f"pair_{i}_left.raw"))
            Rh[i].tofile(os.path.join(d, f"pair_{i}_right.raw"))
        with open(os.path.join(d, "params.txt"), "w") as f:
            f.write(f"{W} {H} {NFEAT} {MBF!r} {mb!r} {B}\n")
        per_k, dig = loop(d, args.dropin_via)
        alt = None
        if args.dropin_via == "frame":
            alt_k, alt_dig = loop(d, "facade")
            alt = {"via": "facade (two ExtractORB threads + ComputeStereoMatches)",
                   "per_trackers": [alt_k[k] for k in ks],
                   "digests_equal_one_call": alt_dig == dig}
            # the same two-thread facade with mvImagePyramid refreshed by every operator()
            # (the host pyramid copy on, as for an unchanged Frame::ComputeStereoMatches):
            # operator()'s added cost
            pyr_k, pyr_dig = loop(d, "pyr")
            alt["host_pyramid"] = {
                "via": "facade, every operator() refreshing mvImagePyramid (pinned host copy of "
                       "the pyramid, ORBextractor.cc:1129-1154), stereo through orbx_stereo_match",
                "per_trackers": [pyr_k[k] for k in ks], "digests_equal_one_call": pyr_dig == dig,
                "added_ms_median_per_frame": {
                    k: pyr_k[k]["latency"]["median_ms"] - alt_k[k]["latency"]["median_ms"]
                    for k in ks}}
    cpu = None
    if args.cpu_seconds > 0:
        cpu = cpu_baseline(pairs, mb, min(args.cpu_seconds, 6.0))
    k0 = per_k[ks[0]]
    lat = k0["latency"]
    via = {"facade": "ORB_SLAM2::ORBextractor facade: Frame::ExtractORB x2 on 2 threads + "
                     "ComputeStereoMatches",
           "frame": "facade, the stereo Frame's extraction + matching as one two-image "
                    "submission (orbx_glue::ExtractStereo)",
           "cabi": "C ABI: orbx_extract x2 on 2 threads + orbx_stereo_match"}[args.dropin_via]
    out = {"metric": f"per-stereo-frame latency of the drop-in host path ({via}), KITTI 1241x376",
           "value": 1000.0 / lat["mean_ms"] if ks[0] == 1 else k0["pairs_per_s"],
           "unit": "frames/sec", "n_gpus": 1,
           "steps": args.frames, "warmup": warm, "ms_per_step": lat["mean_ms"],
           "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic",
           "config": {"workload": "kitti_stereo_dropin_host_path", "width": W, "height": H,
                      "nfeatures": NFEAT, "distinct_pairs": B,
                      "threads_per_tracker": 1 if args.dropin_via == "frame" else 2,
                      "trackers": ks, "via": args.dropin_via,
                      "io": "host images in, host keypoints/descriptors/uRight/depth out"},
           "latency": lat, "mean_keypoints_left": k0["mean_keypoints_left"],
           "mean_stereo_matches": k0["mean_stereo_matches"],
           "per_trackers": [per_k[k] for k in ks], "two_thread_facade": alt, "cpu_baseline": cpu}
    if cpu:
        out["speedup_vs_cpu_median"] = cpu["median_ms"] / lat["median_ms"]
    emit(json.dumps(out))


# ---- configs[0]: one TUM frame, extraction + ComputeBoW + SearchByBoW vs one keyframe --------

TUM_W, TUM_H, TUM_NFEAT = 640, 480, 1000          # Examples/RGB-D/TUM1.yaml:42


def main_tum(args):
    """configs[0] ("Single 640x480 TUM RGB-D frame, 1000 features, ORBextractor + SearchByBoW
    vs one keyframe"), as Tracking::TrackReferenceKeyFrame runs it (Tracking.cc:805-847): per
    frame ExtractORB, Frame::ComputeBoW (DBoW2 transform) and ORBmatcher(0.7, true)
    .SearchByBoW(reference keyframe, frame), on the drop-in host path one frame at a time (the
    C++ loop of tests/native/boundary_test.cpp `tum`).  The vocabulary is synthetic (ORBvoc.txt
    is absent): k = 10, L = 5 with levelsup 3, so FeatureVector buckets sit at level 2 of the
    tree as with ORBvoc's L = 6, levelsup 4.  Beside it the CPU restatement of the same frame
    work on one core (the reference runs it on the Tracking thread)."""
    import subprocess
    import tempfile
    from my_orb_slam2_amd import synth
    P = max(1, min(args.distinct, 16))
    pairs = [synth.stereo_pair(3000 + i, TUM_W, TUM_H) for i in range(P)]
    warm = max(20, args.warmup)
    binp = os.path.join(ROOT, "tests", "native", "boundary_test")
    levelsup = 3
    with tempfile.TemporaryDirectory() as d:
        voc = os.path.join(d, "voc.txt")
        synth.write_vocabulary(voc, k=10, L=5, seed=11)
        for i, (L, R) in enumerate(pairs):
            L.tofile(os.path.join(d, f"pair_{i}_left.raw"))
            R.tofile(os.path.join(d, f"pair_{i}_right.raw"))
        with open(os.path.join(d, "params.txt"), "w") as f:
            f.write(f"{TUM_W} {TUM_H} {TUM_NFEAT} {P} {levelsup} {voc}\n")
        r = subprocess.run([binp, "tum", d, str(args.frames), str(warm)], capture_output=True,
                           text=True, timeout=600)
        if r.returncode != 0:
            sys.exit(f"bench.py: {binp} tum failed ({r.returncode}): {r.stderr[-2000:]}")
        res = json.loads(r.stdout.strip().splitlines()[-1])
        cpu = None
        if args.cpu_seconds > 0:
            import oracle
            from oracle import matcher as om
            from my_orb_slam2_amd.features import FeatureSet, FeatureVector
            ov = om.OracleVocabulary(voc)
            rng = np.random.default_rng(0)
            kfs = []
            for L, _ in pairs:
                k, dsc = oracle.OracleExtractor(TUM_NFEAT, 1.2, 8, 20, 7)(L)
                fv = FeatureVector(*ov.transform(dsc, levelsup)[3])
                kfs.append((FeatureSet(k, dsc, None, fv, None), rng.random(len(k)) < 0.85))
            ox = oracle.OracleExtractor(TUM_NFEAT, 1.2, 8, 20, 7)
            ms, t_end, f = [], time.perf_counter() + min(args.cpu_seconds, 10.0), 0
            while time.perf_counter() < t_end or len(ms) < 20:
                i = f % P
                t0 = time.perf_counter()
                k, dsc = ox(pairs[i][1])
                fv = FeatureVector(*ov.transform(dsc, levelsup)[3])
                om.search_by_bow_kf_frame(kfs[i][0], kfs[i][1], FeatureSet(k, dsc, None, fv, None),
                                          0.7, True)
                t1 = time.perf_counter()
                f += 1
                if f > warm // 4:
                    ms.append(1000.0 * (t1 - t0))
            cpu = {"value": 1000.0 / float(np.mean(ms)), "unit": "frames/sec", "cores": 1,
                   "kind": "port", "sample": f"{len(ms)} TUM-size synthetic frames: extraction + "
                   "DBoW2 transform + SearchByBoW(KF, F) restatement, one thread",
                   **latency_stats(ms)}
    lat = latency_stats(res["latency_ms"])
    out = {"metric": "configs[0] per-frame latency: TUM 640x480 extract + ComputeBoW + "
                     "SearchByBoW vs one keyframe (drop-in host path)",
           "value": 1000.0 / lat["mean_ms"], "unit": "frames/sec", "n_gpus": 1,
           "steps": args.frames, "warmup": warm, "ms_per_step": lat["mean_ms"],
           "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic",
           "config": {"workload": "tum_extract_bow_searchbybow", "width": TUM_W,
                      "height": TUM_H, "nfeatures": TUM_NFEAT, "nnratio": 0.7,
                      "check_orientation": True, "vocabulary": "synthetic k=10 L=5",
                      "levelsup": levelsup, "distinct_frames": P},
           "latency": lat, "mean_keypoints": res["mean_keypoints"],
           "mean_bow_matches": res["mean_bow_matches"], "cpu_baseline": cpu}
    if cpu:
        out["speedup_vs_cpu_median"] = cpu["median_ms"] / lat["median_ms"]
    emit(json.dumps(out))


# ---- keyframe database candidate detection --------------------------------

def main_kfdb(args):
    """KeyFrameDatabase::DetectRelocalizationCandidates (KeyFrameDatabase.cc:220-337), the step
    before configs[3]'s SearchByBoW loop (Tracking.cc:1447-1461), on a --kfs keyframe database
    resident in HBM (synthetic BowVectors of ~300 words, 10 covisibles per keyframe).  One step
    = one query frame: upload of its BowVector, the database scan, the selection, the
    candidate list back on the host."""
    from my_orb_slam2_amd import KeyFrameDatabase, synth
    n = args.kfs
    bows, cov, _ = synth.kfdb_scene(21, n_kf=n, revisit=n // 20)
    db = KeyFrameDatabase(10)
    for b in bows:
        db.add(b)
    for s, nb in enumerate(cov):
        db.set_covisibles(s, nb)
    rng = np.random.default_rng(5)
    queries = [synth.kfdb_query(100 + q, bows[int(rng.integers(0, n))],
                                keep=0.8 if q % 2 == 0 else 0.35) for q in range(64)]
    for q in range(args.warmup):
        db.DetectRelocalizationCandidates(queries[q % len(queries)])
    scan, sel, ncand, wall = [], [], [], []
    for q in range(args.steps):
        t0 = time.perf_counter()
        c = db.DetectRelocalizationCandidates(queries[q % len(queries)])
        wall.append(1000.0 * (time.perf_counter() - t0))
        a, b = db.last_timing()
        scan.append(a)
        sel.append(b)
        ncand.append(len(c))
    entries = sum(len(b[0]) for b in bows)
    scan_ms = float(np.mean(scan))
    scan_bytes = entries * 12 + n * 13          # words + weights, offsets / alive / outputs
    cpu = None
    if args.cpu_seconds > 0:
        from oracle.kfdb import OracleKeyFrameDatabase
        o = OracleKeyFrameDatabase(10)
        for b in bows:
            o.add(b)
        for s, nb in enumerate(cov):
            o.set_covisibles(s, nb)
        ms, t_end = [], time.perf_counter() + min(args.cpu_seconds, 10.0)
        while time.perf_counter() < t_end or len(ms) < 5:
            t0 = time.perf_counter()
            o.DetectRelocalizationCandidates(queries[len(ms) % len(queries)])
            ms.append(1000.0 * (time.perf_counter() - t0))
        cpu = {"value": 1000.0 / float(np.mean(ms)), "unit": "queries/sec", "cores": 1,
               "kind": "port", "sample": f"{len(ms)} queries of the restated KeyFrameDatabase "
               f"(inverted file, oracle/orb_kfdb_oracle.cpp) on {n} keyframes",
               **latency_stats(ms)}
    out = {"metric": f"DetectRelocalizationCandidates queries/sec, {n}-keyframe database",
           "value": 1000.0 / float(np.mean(wall)), "unit": "queries/sec", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": float(np.mean(wall)),
           "higher_is_better": True, "scaling": "none", "vs_baseline": None,
           "dtype": "f64 (DBoW2 weights)", "data": "synthetic",
           "config": {"workload": "kfdb_relocalisation_candidates", "keyframes": n,
                      "bow_entries": entries, "covisibles": 10},
           "latency": latency_stats(wall), "mean_candidates": float(np.mean(ncand)),
           "kernel_ms": {"k_kfdb_scan": scan_ms, "k_kfdb_select": float(np.mean(sel))},
           "roofline": {"kernel": "k_kfdb_scan", "bound": "hbm",
                        "achieved": scan_bytes / (scan_ms / 1000.0) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": scan_bytes / (scan_ms / 1000.0) / 1e9 / HBM_PEAK_GBS,
                        "algorithmic_bytes_per_launch": scan_bytes, "traffic": None},
           "cpu_baseline": cpu}
    emit(json.dumps(out))


# ---- EuRoC mono tracking (configs[2]) ----------------------------------------------------------

EUROC_W, EUROC_H, EUROC_NFEAT = 752, 480, 1000     # Examples/Monocular/EuRoC.yaml


def main_euroc(args):
    """configs[2]: per frame, ORBextractor (1000 features) + UndistortKeyPoints +
    AssignFeaturesToGrid + SearchLocalPoints (Tracking.cc:1297-1347): Frame::isInFrustum +
    MapPoint::PredictScale on each of `--queries` local MapPoints, then SearchByProjection
    (Frame, local MapPoints).  The local maps (poses, MapPoint positions / normals /
    distances / descriptors) and the motion-model claims are inputs resident in HBM; B
    frames per step on one stream."""
    import torch
    import torch.distributed as dist
    from my_orb_slam2_amd import synth
    from my_orb_slam2_amd.tracking import MonoTrackBatch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # ORBX_FORCE_DIST=1 takes the process-group path at world size 1 (torchrun
    # --nproc-per-node 1), so the RCCL timing path can be exercised on a one-GPU box
    dist_on = world > 1 or (os.environ.get("ORBX_FORCE_DIST") == "1" and "RANK" in os.environ)
    if dist_on:   # bound to this rank's GPU, so RCCL's barrier never guesses the device
        dist.init_process_group("nccl", init_method="env://", device_id=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    K4, distc = synth.EUROC_CAM
    B = args.batch or 256
    P = max(1, min(args.distinct, B))
    frames, idx = euroc_frames(rank, B, P)
    d_imgs = torch.from_numpy(np.stack([frames[i] for i in idx])).to(dev)
    mt = MonoTrackBatch(B, EUROC_W, EUROC_H, K4, distc, EUROC_NFEAT, device=local)
    if args.overlap is not None:
        mt.ext.set_overlap(*[int(v) for v in args.overlap.split(",")])

    # inputs: each frame's 3-D local map (built from the frame's own features), projected
    # into the frame inside the step (isInFrustum + PredictScale on the device)
    mt.frames(d_imgs, st)
    nkp, ku, desc = mt.fetch_undistorted()
    per = euroc_local_maps(idx, nkp, ku, desc, args.queries, mt.kp_cap, mt.bounds)
    inp = euroc_device_inputs(torch, dev, per, idx)
    q_off_h = inp["q_off_h"]
    out = torch.empty(int(q_off_h[-1]), dtype=torch.int32, device=dev)
    cnt = torch.empty(B, dtype=torch.int32, device=dev)
    lmap = (inp["frames"], inp["mps"], inp["max_mps"], inp["skip"], inp["nvis"], 1.0)

    def step():
        mt(d_imgs, inp["desc"], inp["q"], inp["q_off"], out, cnt, inp["claimed"], st,
           local_map=lmap)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    mt.matcher.sync(st)
    prof_on = not args.no_kernel_timing
    mt.ext.profile(prof_on)
    mt.matcher.profile(prof_on)
    mt.ext.collect_profile()
    mt.matcher.collect_profile()
    if dist_on:
        dist.barrier(device_ids=[local])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier(device_ids=[local])
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    mt.matcher.sync(st)
    prof = {}
    if prof_on:
        prof.update(mt.ext.collect_profile())
        prof.update({k: v for k, v in mt.matcher.collect_profile().items() if v[1]})
    counts = cnt.cpu().numpy()
    nvis = inp["nvis"].cpu().numpy()
    roof = None
    if prof:
        # the largest kernel group of the step (one stream, one batch: the launches do not
        # overlap), against the HBM roof like the headline's
        gt = split_level(prof)
        geo = step_bytes(mt.ext, B, 0)
        kc = mt.kp_cap
        nq = int(q_off_h[-1])
        # window search: query (16 B record + 32 B descriptor) in, the grid cells of the
        # window and the candidates' keypoints + descriptors (L2-resident) counted once per
        # frame, 16 B top-2 out per query
        geo["k_proj_search"] = nq * (48 + 16) + B * (kc * (28 + 32) + 4 * 3073)
        cand = {k: v for k, v in gt.items() if k in HEADLINE_GROUPS + ("k_proj_search",
                                                                      "k_proj_resolve")}
        dom = max(cand, key=lambda k: cand[k][0])
        roof = roofline_entry(dom, *gt[dom], args.steps, geo.get(dom),
                              traffic_per_step(args.traffic_csv, dom))
        roof["selected_by"] = "largest kernel group per step (one stream)"
        roof["kernel_ms_per_step"] = {k: round(v[0] / max(args.steps, 1), 4)
                                      for k, v in gt.items()}
        roof["valu"] = valu_entry(args.insts_csv, dom, roof["avg_launch_ms"] / 1000.0,
                                  ONE_STREAM_LAUNCHES.get(dom, 1) / roof["launches_per_step"])
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = euroc_cpu_baseline(frames, [per[p] for p in range(P)], args.cpu_seconds)
    if rank == 0:
        out_line = {"metric": "frames/sec ORB extract + SearchByProjection vs 20-KF local map, "
                              "EuRoC 752x480 mono",
                    "value": B * args.steps * world / elapsed, "unit": "frames/sec",
                    "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                    "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
                    "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
                    "config": {"workload": "euroc_mono_extract_search_local_points",
                               "width": EUROC_W, "height": EUROC_H, "nfeatures": EUROC_NFEAT,
                               "queries_per_frame": args.queries, "nnratio": 0.8, "th": 1.0,
                               "frames_per_step_per_gpu": B, "distinct_frames": P,
                               "parallelism": f"dp{world}"},
                    "mean_keypoints": float(nkp.mean()),
                    "mean_local_map_matches": float(counts.mean()),
                    "mean_local_map_points_in_view": float(nvis.mean()),
                    "roofline": roof, "cpu_baseline": cpu}
        emit(json.dumps(out_line))
    if dist_on:
        dist.destroy_process_group()


def euroc_cpu_baseline(frames, inputs, budget_s):
    """The CPU restatement of the same per-frame work on one host core: extraction,
    undistortion, grid and the projection search (Tracking runs them on one thread)."""
    try:
        import oracle
        from oracle import matcher as om
    except Exception:
        return None
    from my_orb_slam2_amd import synth
    from my_orb_slam2_amd.features import (PROJ_FRAME_MAPPOINTS, PROJ_QUERY_DTYPE, FeatureSet,
                                           assign_features_to_grid)
    K4, distc = synth.EUROC_CAM
    bounds = None
    ox = oracle.OracleExtractor(EUROC_NFEAT, 1.2, 8, 20, 7)
    done, t0 = 0, time.perf_counter()
    while True:
        p = done % len(frames)
        k, d = ox(frames[p])
        un = om.undistort_keypoints(k, K4, distc)
        if bounds is None:
            bounds = om.image_bounds(K4, distc, EUROC_W, EUROC_H)
        ku = k.copy()
        ku["x"], ku["y"] = un[:, 0], un[:, 1]
        g = assign_features_to_grid(ku, *bounds)
        pose, mps, qd, skip, cl = inputs[p]
        qb, _ = om.is_in_frustum(pose, mps, skip, 0.5, 1.0)
        q = qb.view(PROJ_QUERY_DTYPE)
        om.search_by_projection(PROJ_FRAME_MAPPOINTS, FeatureSet(ku, d, None, None, g), q, qd,
                                cl[:len(k)], None, nnratio=0.8)
        done += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "frames/sec", "cores": 1, "kind": "port",
            "sample": f"{done} EuRoC-size synthetic frames: extraction + undistort + grid + "
                      f"isInFrustum / PredictScale + SearchByProjection restatement, one "
                      f"thread, {el:.1f} s",
            "host_cpus": os.cpu_count()}


# ---- matcher workloads (configs[3], configs[4]) ----------------------------------------------

VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12   # 256 CUs x 128 lane-ops/clk x 2.4 GHz (guide)
# Measured issue cost on gfx950 (profiles/r01_valu_issue_rates.txt): v_xor_b32 issues at 2
# cycles per wave64 instruction, v_bcnt_u32_b32 at 4; a 256-bit distance is 8 of each, so one
# SIMD retires at most 64 distances per 48 cycles.
DIST_ISSUE_PEAK = 1024 * 2.4e9 * 64 / 48
# Dense int8 matrix peak (MI355X_MICROARCH.md §Matrix cores: i8 = 2x the bf16 rate, bf16 ~2.5
# PFLOP/s dense): v_mfma_i32_32x32x32_i8, the k_bf_mfma distances
I8_MFMA_PEAK_TOPS = 5000.0


def _hash_bytes(torch, idx, salt):
    """Deterministic pseudo-random bytes of global indices (same on every rank)."""
    x = idx * 6364136223846793005 + (1442695040888963407 + salt)
    x = x ^ (x >> 29)
    x = x * -49064778989728563
    x = x ^ (x >> 32)
    return x


def _reloc_db(torch, dev, k0, k1, F):
    """Keyframes [k0, k1) of the synthetic relocalisation database: F features each, one
    FeatureVector node per keyframe (the brute-force anchor of SURVEY §8c), 90 % of the
    features with a valid MapPoint."""
    from my_orb_slam2_amd.matcher import KfDbC
    K = k1 - k0
    g = torch.arange(k0 * F, k1 * F, device=dev, dtype=torch.int64)
    words = _hash_bytes(torch, g[:, None] * 8 + torch.arange(8, device=dev), 0)
    desc = (words & 0xFFFFFFFF).to(torch.int32).contiguous().view(torch.uint8).reshape(-1, 32)
    keys = torch.zeros(K * F, 7, dtype=torch.float32, device=dev)
    keys[:, 3] = (_hash_bytes(torch, g, 77) & 0xFFFF).to(torch.float32) * (360.0 / 65536.0)
    flag = ((_hash_bytes(torch, g, 99) & 1023) < 922).to(torch.uint8)
    feat_off = (torch.arange(K + 1, device=dev, dtype=torch.int32) * F).contiguous()
    node_off = torch.arange(K + 1, device=dev, dtype=torch.int32)
    node_id = torch.zeros(max(K, 1), dtype=torch.int32, device=dev)
    node_feat = torch.arange(F, device=dev, dtype=torch.int32).repeat(K).contiguous()
    keep = [desc, keys, flag, feat_off, node_off, node_id, node_feat]
    c = KfDbC(K, F, feat_off.data_ptr(), keys.data_ptr(), desc.data_ptr(), 0, flag.data_ptr(),
              node_off.data_ptr(), node_id.data_ptr(), feat_off.data_ptr(), node_feat.data_ptr())
    return c, keep, int(flag.sum().item())


def _reloc_query(torch, dev, n_kfs, F, seed=5):
    """The query frame: 30 % of its descriptors are noisy copies of 30 features from each of
    10 database keyframes (so those keyframes pass the >= 15 match test), the rest random."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    true_kfs = torch.randperm(n_kfs, generator=g)[:10]
    src = (true_kfs[:, None] * F + torch.randint(0, F, (10, 30), generator=g)).reshape(-1)
    n_copy = src.numel()
    rnd = torch.randint(0, 2**31, (F - n_copy, 8), generator=g, dtype=torch.int64)
    words = torch.cat([_hash_bytes(torch, src[:, None] * 8 + torch.arange(8), 0), rnd])
    desc = (words & 0xFFFFFFFF).to(torch.int32).contiguous().view(torch.uint8).reshape(-1, 32)
    flips = torch.randint(0, 256, (n_copy, 20), generator=g)
    keepflip = torch.rand(n_copy, 20, generator=g) < torch.rand(n_copy, 1, generator=g)
    for i in range(n_copy):
        for b in flips[i][keepflip[i]].tolist():
            desc[i, b // 8] ^= (1 << (b % 8))
    keys = torch.zeros(F, 7, dtype=torch.float32)
    ang = (_hash_bytes(torch, src, 77) & 0xFFFF).to(torch.float32) * (360.0 / 65536.0)
    keys[:n_copy, 3] = torch.remainder(ang - 20.0 + torch.randn(n_copy, generator=g), 360.0)
    keys[n_copy:, 3] = torch.rand(F - n_copy, generator=g) * 360.0
    return desc.to(dev), keys.to(dev), true_kfs


def main_match(args):
    import torch
    import torch.distributed as dist
    from my_orb_slam2_amd import ORBmatcher
    from my_orb_slam2_amd.distributed import (all_gather_counts, broadcast_query,
                                              gather_candidate_blocks, gather_rows, shard_range)
    from my_orb_slam2_amd.features import FeatureSetC

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # ORBX_FORCE_DIST=1 takes the process-group path at world size 1 (torchrun
    # --nproc-per-node 1), so the RCCL timing path can be exercised on a one-GPU box
    dist_on = world > 1 or (os.environ.get("ORBX_FORCE_DIST") == "1" and "RANK" in os.environ)
    if dist_on:   # bound to this rank's GPU, so RCCL's barrier never guesses the device
        dist.init_process_group("nccl", init_method="env://", device_id=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    # every rank must own at least one unit, or its shard structures are empty while the
    # other ranks wait in the collectives
    units_total = args.kfs if args.workload == "reloc" else args.jobs
    if units_total < world:
        sys.exit(f"bench.py: {units_total} {'keyframes' if args.workload == 'reloc' else 'jobs'}"
                 f" < world size {world}")

    if args.workload == "reloc":
        F = 1000
        k0, k1 = shard_range(args.kfs, rank, world)
        db, keep, nvalid = _reloc_db(torch, dev, k0, k1, F)
        qdesc, qkeys, true_kfs = _reloc_query(torch, dev, args.kfs, F)
        qn_off = torch.tensor([0, F], dtype=torch.int32, device=dev)
        q_node = torch.zeros(1, dtype=torch.int32, device=dev)
        q_feat = torch.arange(F, dtype=torch.int32, device=dev)
        fc = FeatureSetC()
        fc.n, fc.keys, fc.desc = F, qkeys.data_ptr(), qdesc.data_ptr()
        fc.n_nodes, fc.node_id, fc.node_off, fc.node_feat = (1, q_node.data_ptr(),
                                                            qn_off.data_ptr(), q_feat.data_ptr())
        m = ORBmatcher(0.75, True, device=local)      # Tracking.cc:1461
        out = torch.empty((k1 - k0, F), dtype=torch.int32, device=dev)
        cnt = torch.empty(max(k1 - k0, 1), dtype=torch.int32, device=dev)

        def step():
            if dist_on:
                broadcast_query([qdesc, qkeys])
            m.search_by_bow_kf_frame_batch_device(db, fc, out, cnt, st)
            if dist_on:
                allc = all_gather_counts(cnt[:k1 - k0], args.kfs, world)
                # the candidates' match lists travel to every rank (Tracking.cc:1503-1528), built
                # and exchanged on the device: no host round trip inside the step
                gather_candidate_blocks(out, cnt[:k1 - k0], k0, world)
                return allc
            return cnt[:k1 - k0]
        units, unit_name = 1, "query frames/sec"
        work_ops = 16.0 * nvalid * F                   # 8 XOR + 8 BCNT per distance
        hbm_bytes = float((k1 - k0) * F * (32 + 4 + 1) + F * (32 + 28))
        kern = "k_bow"
        cfg = {"workload": "relocalisation_bf_vs_keyframes", "keyframes": args.kfs,
               "features_per_keyframe": F, "query_features": F, "nnratio": 0.75,
               "check_orientation": True, "featurevector": "single node (brute force)",
               "parallelism": f"keyframe shards x{world}, RCCL broadcast + all-gather of counts and candidate match lists"}
        metric = "relocalisation query frames/sec, 1000-descriptor frame vs 10k keyframes"
    else:
        from my_orb_slam2_amd import synth
        from my_orb_slam2_amd.matcher import DeviceKfDb
        j0, j1 = shard_range(args.jobs, rank, world)
        kfs, flags, F12, epi = triangulation_jobs(j0, j1)
        db = DeviceKfDb(kfs, flags, dev)
        nj = j1 - j0
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        kf1 = T(np.arange(nj, dtype=np.int32) * 2)
        kf2 = T(np.arange(nj, dtype=np.int32) * 2 + 1)
        n1 = np.array([kfs[2 * i].n for i in range(nj)], np.int32)
        job_off = T(np.concatenate([[0], np.cumsum(n1)]).astype(np.int32))
        dF, dE = T(np.array(F12, np.float32)), T(np.array(epi, np.float32))
        s, s2, _ = synth.scale_tables()
        m = ORBmatcher(0.6, False, device=local)      # LocalMapping.cc:276
        # the resident database in node order (built with it, like the upload; not timed):
        # the kernel reads each vocabulary node's features as contiguous runs
        if not args.tri_gather:
            db.node_order(m, st)
            torch.cuda.synchronize(dev)
        out = torch.empty(int(n1.sum()), dtype=torch.int32, device=dev)
        cnt = torch.empty(max(nj, 1), dtype=torch.int32, device=dev)

        # whether the match12 arrays are gathered must be decided the same way on every
        # rank (each rank makes the same collective calls): rows gather only when every job
        # of every shard has the same KF1 feature count
        row_len = int(n1[0])
        uniform = bool((n1 == row_len).all())
        if dist_on:
            agree = torch.tensor([int(uniform), row_len, -row_len], dtype=torch.int64, device=dev)
            dist.all_reduce(agree, op=dist.ReduceOp.MIN)
            uniform = bool(agree[0].item()) and int(agree[1].item()) == -int(agree[2].item())

        def step():
            m.search_for_triangulation_batch_device(db.c, kf1, kf2, dF, dE, s2, s, job_off, out,
                                                    cnt, stream=st)
            if dist_on:
                if uniform:   # every job's match12 array to every rank
                    gather_rows(out.view(nj, -1), args.jobs, world)
                return all_gather_counts(cnt[:nj], args.jobs, world)
            return cnt[:nj]
        units, unit_name = args.jobs, "keyframe-pair jobs/sec"
        work_ops = None
        kern = "k_triangulate"
        cfg = {"workload": "batched_search_for_triangulation", "jobs": args.jobs,
               "features_per_keyframe": 2000, "vocabulary_nodes": 100, "only_stereo": False,
               "check_orientation": False, "db_layout": "gather" if args.tri_gather else "node order",
               "parallelism": f"job shards x{world}, RCCL all-gather of counts and match arrays"}
        metric = "SearchForTriangulation keyframe-pair jobs/sec (512 jobs, 2000 features/KF)"

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize(dev)
    m.sync(st)
    m.profile(not args.no_kernel_timing)
    m.collect_profile()
    if dist_on:
        dist.barrier(device_ids=[local])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier(device_ids=[local])
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    m.sync(st)
    prof = m.collect_profile() if not args.no_kernel_timing else {}
    counts = res.cpu().numpy()
    roof = None
    if prof and prof.get(kern, (0, 0))[1]:
        tot_ms, launches = prof[kern]
        avg_s = tot_ms / 1000.0 / launches
        if work_ops is not None:
            ach = work_ops / avg_s / 1e12
            dps = work_ops / 16 / avg_s   # 16 lane-ops per 256-bit distance
            # the same launch against the HBM roof: the shard's descriptors, FeatureVector
            # entries and flags are streamed once per query (37 B per feature), plus the query
            db_bytes = hbm_bytes
            roof = {"kernel": kern, "bound": "valu", "achieved": ach, "peak": VALU_PEAK_TOPS,
                    "unit": "Tops/s (int32 lane-ops)", "frac": ach / VALU_PEAK_TOPS,
                    "traffic": None, "algorithmic_ops_per_launch": work_ops,
                    "avg_launch_ms": avg_s * 1000.0,
                    "distances_per_s": dps,
                    "issue_peak_distances_per_s": DIST_ISSUE_PEAK,
                    "issue_frac": dps / DIST_ISSUE_PEAK,
                    "hbm": {"achieved": db_bytes / avg_s / 1e9, "unit": "GB/s",
                            "peak": HBM_PEAK_GBS,
                            "frac": db_bytes / avg_s / 1e9 / HBM_PEAK_GBS,
                            "algorithmic_bytes_per_launch": db_bytes,
                            **pmc_hbm(args.traffic_csv, kern, avg_s)}}
            roof["traffic"] = roof["hbm"]["traffic"]
        else:
            nbytes = float(sum(fs.n for fs in kfs) * (32 + 28 + 4 + 1))
            ach = nbytes / avg_s / 1e9
            pm = pmc_hbm(args.traffic_csv, kern, avg_s)
            roof = {"kernel": kern, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": pm["traffic"],
                    "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": avg_s * 1000.0,
                    "pmc": pm}
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = match_cpu_baseline(args, torch, keep if args.workload == "reloc" else None,
                                 (qdesc, qkeys) if args.workload == "reloc" else None,
                                 None if args.workload == "reloc" else (kfs, flags, F12, epi))
    if rank == 0:
        extra = {}
        if args.workload == "reloc":
            from my_orb_slam2_amd.distributed import relocalisation_candidates
            cand = relocalisation_candidates(counts)
            extra = {"candidates_ge_15": int(len(cand)),
                     "true_keyframes_found": int(np.isin(true_kfs.numpy(), cand).sum())
                     if world > 1 or args.kfs == k1 - k0 else None}
        else:
            extra = {"mean_pairs_per_job": float(counts.mean())}
        out_line = {"metric": metric, "value": units * args.steps / elapsed, "unit": unit_name,
                    "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                    "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
                    "scaling": "strong", "vs_baseline": None, "dtype": "u8 (256-bit Hamming)",
                    "data": "synthetic", "config": cfg, **extra, "roofline": roof,
                    "cpu_baseline": cpu}
        emit(json.dumps(out_line))
    if dist_on:
        dist.destroy_process_group()


def bf_rows(r0: int, r1: int) -> np.ndarray:
    """Database rows [r0, r1) of the bf workload: 32 bytes per row from a counter hash
    (splitmix64 of 4 * row + k), so any row, and any shard, is computed independently of the
    others and of the world size (uniform random bits)."""
    x = (np.arange(r0, r1, dtype=np.uint64)[:, None] * np.uint64(4) +
         np.arange(4, dtype=np.uint64)[None, :])
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return np.ascontiguousarray(x).view(np.uint8).reshape(r1 - r0, 32)


def bf_query(ndb: int, nq: int = 1000, seed: int = 7):
    """The bf workload's query frame: nq random descriptors, 30 % of them replaced by database
    rows with 0-40 bits flipped.  Returns (q, planted query ids, their rows)."""
    rng = np.random.default_rng(seed)
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    ids = rng.choice(nq, int(0.3 * nq), replace=False)
    rows = rng.integers(0, ndb, len(ids))
    for i, r in zip(ids, rows):
        q[i] = bf_rows(int(r), int(r) + 1)[0]
        for b in rng.choice(256, int(rng.integers(0, 41)), replace=False):
            q[i, b // 8] ^= np.uint8(1 << (b % 8))
    return q, ids, rows


BF_KERNELS = {"mfma": "k_bf_mfma", "valu": "k_bf_top2"}
BF_KERNEL_IDS = {"mfma": 0, "valu": 1}      # ORBX_BF_MFMA / ORBX_BF_VALU (include/orbx_match.h)


def pmc_hbm(traffic_csv, kernel, avg_s):
    """PMC HBM traffic of one launch of `kernel` (FETCH_SIZE x 2 + WRITE_SIZE from the passes
    in traffic_csv, MI355X_MICROARCH.md §HBM) and the rate it gives over the launch's HIP-event
    duration, or Nones when no pass holds the kernel."""
    tr = traffic_from_csv(traffic_csv, kernel)
    if not tr or avg_s <= 0:
        return {"traffic": None, "traffic_GBs": None, "traffic_frac": None}
    return {"traffic": tr, "traffic_GBs": tr / avg_s / 1e9, "traffic_frac": tr / avg_s / 1e9 / HBM_PEAK_GBS}


def bf_roofline(kname, prof, nq, nrows, traffic_csv):
    """Roofline of one brute-force top-2 launch pair (the distance kernel + k_bf_merge, one
    timer interval): k_bf_mfma against the dense i8 matrix peak (256 multiply-adds per
    distance), k_bf_top2 against the int32 lane-op roof (8 XOR + 8 BCNT per distance); both
    against the XOR + BCNT issue roof and HBM (the shard's rows read once per query frame:
    algorithmic bytes; PMC traffic of the distance kernel from traffic_csv)."""
    if not prof or not prof.get("k_bf", (0, 0))[1]:
        return None
    tot_ms, launches = prof["k_bf"]
    avg_s = tot_ms / 1000.0 / launches
    dist_n = float(nq) * nrows
    dps = dist_n / avg_s
    db_bytes = 32.0 * nrows + 32.0 * nq + 12.0 * nq
    if kname == "k_bf_mfma":
        ops = 512.0 * dist_n
        unit, peak, bound = "TOPS (int8 MFMA)", I8_MFMA_PEAK_TOPS, "mfma"
    else:
        ops = 16.0 * dist_n
        unit, peak, bound = "Tops/s (int32 lane-ops)", VALU_PEAK_TOPS, "valu"
    hbm = {"achieved": db_bytes / avg_s / 1e9, "unit": "GB/s", "peak": HBM_PEAK_GBS,
           "frac": db_bytes / avg_s / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": db_bytes}
    pm = pmc_hbm(traffic_csv, kname, avg_s)
    hbm.update(pm)
    return {"kernel": kname + " + k_bf_merge", "bound": bound, "achieved": ops / avg_s / 1e12,
            "peak": peak, "unit": unit, "frac": ops / avg_s / 1e12 / peak,
            "traffic": pm["traffic"], "algorithmic_ops_per_launch": ops,
            "avg_launch_ms": avg_s * 1000.0, "distances_per_s": dps,
            "issue_peak_distances_per_s": DIST_ISSUE_PEAK, "issue_frac": dps / DIST_ISSUE_PEAK,
            "hbm": hbm}


def main_bf(args):
    """configs[3] as a pure brute-force top-2: one query frame (1000 descriptors) against the
    whole descriptor database (default 10^7 rows = 10k keyframes x 1000), the rows sharded
    across ranks.  Step: RCCL broadcast of the query (32 KB), every rank's top-2 over
    its shard (orbx_hamming_bf_top2_device, global row numbers), RCCL all-gather of the
    12-byte per-query results and the merge in rank order (distributed.gather_top2)."""
    import torch
    import torch.distributed as dist

    from my_orb_slam2_amd import ORBmatcher, load
    from my_orb_slam2_amd.distributed import broadcast_query, gather_top2, shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_on = world > 1 or (os.environ.get("ORBX_FORCE_DIST") == "1" and "RANK" in os.environ)
    if dist_on:
        dist.init_process_group("nccl", init_method="env://", device_id=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    ndb = args.db_rows
    if ndb < world:
        sys.exit(f"bench.py: {ndb} database rows < world size {world}")
    r0, r1 = shard_range(ndb, rank, world)
    ddb = torch.empty((r1 - r0, 32), dtype=torch.uint8, device=dev)
    blk = 1 << 20
    for b0 in range(r0, r1, blk):                  # the shard, built block by block
        b1 = min(b0 + blk, r1)
        ddb[b0 - r0:b1 - r0] = torch.from_numpy(bf_rows(b0, b1)).to(dev)
    qh, ids, rows = bf_query(ndb)
    nq = len(qh)
    dq = torch.from_numpy(qh).to(dev)
    m = ORBmatcher(0.75, True, device=local)
    m.set_bf_kernel(BF_KERNEL_IDS[args.bf_kernel])
    out = [torch.empty(nq, dtype=torch.int32, device=dev) for _ in range(3)]

    def step():
        if dist_on:
            broadcast_query([dq])
        m.hamming_bf_top2_device(dq, nq, ddb, r1 - r0, *out, idx_base=r0, stream=st)
        if dist_on:
            return gather_top2(*out, world)
        return out

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize(dev)
    m.profile(not args.no_kernel_timing)
    m.collect_profile()
    if dist_on:
        dist.barrier(device_ids=[local])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier(device_ids=[local])
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = m.collect_profile() if not args.no_kernel_timing else {}
    bi, bd, sd = (t.cpu().numpy() for t in res)
    kname = BF_KERNELS[args.bf_kernel]
    roof = bf_roofline(kname, prof, nq, r1 - r0, args.traffic_csv)
    # north_star's kernel beside the default: the other distance kernel timed on the same
    # inputs after the timed region (same steps, same collectives), its results compared
    alt = None
    if not args.no_kernel_timing:
        akey = "valu" if args.bf_kernel == "mfma" else "mfma"
        m.set_bf_kernel(BF_KERNEL_IDS[akey])
        for _ in range(2):
            res_a = step()
        torch.cuda.synchronize(dev)
        m.collect_profile()
        if dist_on:
            dist.barrier(device_ids=[local])
        t1 = time.perf_counter()
        for _ in range(args.steps):
            res_a = step()
        torch.cuda.synchronize(dev)
        if dist_on:
            dist.barrier(device_ids=[local])
        el_a = time.perf_counter() - t1
        if dist_on:
            t = torch.tensor([el_a], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_a = float(t.item())
        prof_a = m.collect_profile()
        same = all(bool(torch.equal(x, y)) for x, y in zip(res_a, res))
        alt = {"kernel": BF_KERNELS[akey], "value": args.steps / el_a, "unit": "query frames/sec",
               "ms_per_step": 1000.0 * el_a / args.steps, "outputs_equal_default": same,
               "roofline": bf_roofline(BF_KERNELS[akey], prof_a, nq, r1 - r0, args.traffic_csv)}
        m.set_bf_kernel(BF_KERNEL_IDS[args.bf_kernel])
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        try:
            from oracle import matcher as om
            n_s, spent = 2000, 0.0
            while spent < min(args.cpu_seconds, 20.0) / 4 and n_s < ndb:
                t1 = time.perf_counter()
                om.bf_top2(qh, bf_rows(0, n_s))
                spent = time.perf_counter() - t1
                if spent < min(args.cpu_seconds, 20.0) / 4:
                    n_s = min(ndb, n_s * 4)
            per_frame = spent * ndb / n_s
            cpu = {"value": 1.0 / per_frame, "unit": "query frames/sec", "cores": 1,
                   "kind": "port",
                   "sample": f"the 1000-descriptor query frame against {n_s} of the {ndb} rows "
                             f"({spent:.1f} s, oracle_bf_top2: ORBmatcher's best / second loop), "
                             f"scaled to the whole database"}
        except Exception:
            cpu = None
    if rank == 0:
        found = int((bi[ids] == rows).sum())
        line = {"metric": "brute-force top-2 query frames/sec, 1000 descriptors vs "
                          f"{ndb} database descriptors", "value": args.steps / elapsed,
                "unit": "query frames/sec", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                "dtype": "u8 (256-bit Hamming)", "data": "synthetic",
                "config": {"workload": "relocalisation_pure_bf_top2", "db_rows": ndb,
                           "query_descriptors": nq, "planted_queries": int(len(ids)),
                           "parallelism": f"row shards x{world}, RCCL broadcast + all-gather "
                                          "of per-query top-2, merge in rank order"},
                "planted_found": found, "mean_best_dist": float(bd.mean()),
                "roofline": roof, "alt_kernel": alt, "cpu_baseline": cpu}
        emit(json.dumps(line))
    if dist_on:
        dist.destroy_process_group()


def match_cpu_baseline(args, torch, db_keep, query, tri):
    """The matcher restatement (oracle/) timed on one host core over a bounded sample of the
    same workload, scaled to the workload's unit."""
    try:
        from oracle import matcher as om
    except Exception:
        return None
    from my_orb_slam2_amd._lib import KEYPOINT_DTYPE
    from my_orb_slam2_amd.features import FeatureSet, feature_vector
    budget = min(args.cpu_seconds, 20.0)
    done, t0 = 0, time.perf_counter()
    if db_keep is not None:
        desc, keys, flag = (t.cpu().numpy() for t in db_keep[:3])
        F = 1000
        qd, qk = (t.cpu().numpy() for t in query)

        def fs(d, k):
            kp = np.zeros(len(d), KEYPOINT_DTYPE)
            kp["angle"] = k[:, 3]
            return FeatureSet(kp, d, None, feature_vector(np.zeros(len(d))), None)
        frame = fs(qd, qk)
        nkf = len(desc) // F
        while time.perf_counter() - t0 < budget and done < nkf:
            sl = slice(done * F, (done + 1) * F)
            om.search_by_bow_kf_frame(fs(desc[sl], keys[sl]), flag[sl], frame, 0.75, True)
            done += 1
        el = time.perf_counter() - t0
        return {"value": done / el / args.kfs, "unit": "query frames/sec", "cores": 1,
                "kind": "port", "sample": f"SearchByBoW(KF, F) restatement on {done} of the "
                f"{args.kfs} keyframes in {el:.1f} s, scaled to the whole database"}
    kfs, flags, F12, epi = tri
    from my_orb_slam2_amd import synth
    s, s2, _ = synth.scale_tables()
    nj = len(F12)
    while time.perf_counter() - t0 < budget and done < nj:
        om.search_for_triangulation(kfs[2 * done], flags[2 * done], kfs[2 * done + 1],
                                    flags[2 * done + 1], F12[done].reshape(3, 3), epi[done], s2,
                                    s, False, False)
        done += 1
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "keyframe-pair jobs/sec", "cores": 1, "kind": "port",
            "sample": f"SearchForTriangulation restatement on {done} of the {nj} jobs, "
                      f"{el:.1f} s"}


if __name__ == "__main__":
    main()
