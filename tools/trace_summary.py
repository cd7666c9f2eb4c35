"""Summaries of a rocprofv3 --hip-trace --kernel-trace run of the drop-in loop
(tools/dropin_trace.sh): one stereo frame's timeline (HIP API calls per thread, kernels per
queue) and, over the middle 60 % of the run, the kernels' union busy time, per-kernel totals and
the HIP API calls' mean durations.

    python tools/trace_summary.py TRACE_DIR
"""
import collections
import csv
import sys


def main(d):
    api = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
    ker = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Queue_Id"],
                 k["Kernel_Name"].split("(")[0].replace("void ", "")) for k in ker)
    stereo = [k for k in ks if "k_stereo" in k[3] and "cut" not in k[3]]
    a, b = stereo[len(stereo) // 5][0], stereo[4 * len(stereo) // 5][0]
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API t" + r["Thread_Id"][-3:],
           r["Function"]) for r in api]
    ev += [(s, e, "K q" + q, n) for s, e, q, n in ks]
    ev.sort()
    s0, s1 = stereo[len(stereo) // 2 - 1][1], stereo[len(stereo) // 2][1]
    print("one frame (us from the previous frame's k_stereo end):")
    for e in ev:
        if s0 <= e[0] <= s1 + 5000:
            print(f"  {(e[0] - s0) / 1e3:8.1f} {(e[1] - s0) / 1e3:8.1f} {(e[1] - e[0]) / 1e3:7.1f} "
                  f"{e[2]:9s} {e[3]}")
    win = [k for k in ks if a <= k[0] < b]
    busy, cur = 0, a
    for s, e, _, _ in win:
        s = max(s, cur)
        if e > s:
            busy += e - s
            cur = max(cur, e)
    nf = sum(1 for k in win if k[3].endswith("k_stereo"))
    print(f"window {(b - a) / 1e3:.1f} us, {nf} stereo frames, kernels busy (union) "
          f"{busy / 1e3:.1f} us, queues {sorted(set(k[2] for k in win))}")
    by = collections.defaultdict(lambda: [0, 0])
    for s, e, _, n in win:
        by[n][0] += 1
        by[n][1] += e - s
    for n, (c, t) in sorted(by.items(), key=lambda x: -x[1][1]):
        print(f"  {n:28s} n={c:5d} avg {t / c / 1e3:7.2f} us  per frame {t / max(nf, 1) / 1e3:7.1f} us")
    fa = collections.defaultdict(lambda: [0, 0])
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if a <= s < b:
            fa[r["Function"]][0] += 1
            fa[r["Function"]][1] += e - s
    print("HIP API calls in the window:")
    for n, (c, t) in sorted(fa.items(), key=lambda x: -x[1][1])[:10]:
        print(f"  {n:26s} n={c:5d} mean {t / c / 1e3:8.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
