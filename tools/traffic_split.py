"""Per-variant HBM traffic of k_level's level-0 and level-1..7 launches from the passes of
tools/var_traffic.sh / tools/l0_sweep.sh (FETCH_SIZE doubled, both KiB; MI355X_MICROARCH §HBM).
usage: python tools/traffic_split.py DIR NAME...   (DIR/f_NAME, DIR/w_NAME)"""
import csv
import glob
import sys

ALG0_R = ALG0_W = 1024 * 1241 * 376                     # level 0 read once, blurred written once
SIZES = [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151), (416, 126), (346, 105)]
A = [w * h * 1024 for w, h in SIZES]
ALG17_R = sum(A[:7]) / 7                                # level l-1 read
ALG17_W = 2 * sum(A[1:]) / 7                            # level l and its blur written


def per_launch(path, pat):
    tot, ids = 0.0, set()
    for p in glob.glob(path):
        for r in csv.DictReader(open(p)):
            if pat in r["Kernel_Name"]:
                tot += float(r["Counter_Value"])
                ids.add(r["Dispatch_Id"])
    return tot / len(ids) * 1024 if ids else float("nan")


d = sys.argv[1]
for v in sys.argv[2:]:
    f0 = 2 * per_launch(f"{d}/f_{v}/run_counter_collection.csv", "k_level_strip<4>")
    w0 = per_launch(f"{d}/w_{v}/run_counter_collection.csv", "k_level_strip<4>")
    f1 = 2 * per_launch(f"{d}/f_{v}/run_counter_collection.csv", "k_level_strip<3>")
    w1 = per_launch(f"{d}/w_{v}/run_counter_collection.csv", "k_level_strip<3>")
    tot = (f0 + w0 + 7 * (f1 + w1)) / 8
    alg = (ALG0_R + ALG0_W + 7 * (ALG17_R + ALG17_W)) / 8
    print(f"{v:8s} L0 fetch {f0 / ALG0_R:.3f} write {w0 / ALG0_W:.3f} | L1-7 fetch {f1 / ALG17_R:.3f} "
          f"write {w1 / ALG17_W:.3f} | k_level traffic/alg {tot / alg:.3f} ({tot / 1e6:.0f} / {alg / 1e6:.0f} MB per launch)")
