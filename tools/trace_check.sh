#!/bin/bash
# The rocprofv3 kernel trace of the headline command (its launches only: no one-stream pass)
# beside bench.py's own HIP-event launch times of the same command.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --no-kernel-timing --serial-steps 0 > $O/trace.log 2>&1 || { echo TRACE FAILED; tail $O/trace.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 0 --serial-steps 0 > $O/bench20.json 2> $O/bench20.err || { echo BENCH FAILED; tail $O/bench20.err; exit 1; }
python - <<PY
import csv, json
rows = list(csv.DictReader(open("$O/trace/run_kernel_stats.csv")))
agg = {}
for r in rows:
    for k in ("k_level", "k_fast", "k_octree", "k_orient_desc", "k_stereo"):
        if k in r["Name"] and not (k == "k_stereo" and "cut" in r["Name"]):
            t, n = agg.get(k, (0.0, 0)); agg[k] = (t + float(r["TotalDurationNs"]), n + int(r["Calls"]))
j = json.load(open("$O/bench20.json"))
print("trace avg ms per launch:", {k: round(t / n / 1e6, 4) for k, (t, n) in agg.items()})
print("bench k_level avg_launch_ms:", round(j["roofline"]["avg_launch_ms"], 4), "frac", round(j["roofline"]["frac"], 4), "value", round(j["value"]))
PY
