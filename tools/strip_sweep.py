"""k_level_strip strip heights per level (ORBX_STRIP_TH), one bench process per setting, on the
GPU box.  usage: python tools/strip_sweep.py [L:h,h,..] ...   (e.g. 3:36,50 5:78)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(ths, quiet=False):
    env = dict(os.environ, ORBX_STRIP_TH=",".join(str(t) for t in ths))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-seconds", "0",
                        "--steps", os.environ.get("SWEEP_STEPS", "200"), "--warmup", "30"], env=env, capture_output=True,
                       text=True, timeout=300)
    if r.returncode != 0:
        print("FAILED", ths, r.stderr[-1500:], flush=True)
        raise SystemExit(1)
    j = json.loads(r.stdout.strip().splitlines()[-1])
    ks = j["roofline"]["kernel_ms_per_step"]
    if not quiet:
        print(f"{env['ORBX_STRIP_TH']:32s} {j['value']:9.0f}/s k_level {ks['k_level']:.4f} "
          f"k_fast {ks['k_fast']:.4f} matches {j.get('mean_stereo_matches')}", flush=True)
    return ks["k_level"]


base = [64] * 8
if sys.argv[1].startswith("base="):
    base = [int(v) for v in sys.argv.pop(1)[5:].split(",")]
# every candidate between two runs of the base (the box's clocks drift over minutes)
for spec in sys.argv[1:]:
    lv, hs = spec.split(":")
    for h in hs.split(","):
        t = list(base)
        t[int(lv)] = int(h)
        b0 = run(base, True)
        c = run(t, True)
        b1 = run(base, True)
        print(f"L{lv} h={h:4s} k_level {c:.4f} vs base {b0:.4f}/{b1:.4f}: {c - (b0 + b1) / 2:+.4f} ms",
              flush=True)
