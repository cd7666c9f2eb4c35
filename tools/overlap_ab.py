"""A/B of the extraction's side branch (orbx_extractor_set_overlap) at run time: bench.py once
per configuration, each in its own process.

    python tools/overlap_ab.py "0" "3,3,1" "3,3,2" ... [-- bench args]   # on the GPU box

Prints one line per configuration: pairs/s, ms per step, per-kernel ms per step (HIP-event
spans: with a side branch they overlap), the one-stream pass of the same run."""
from __future__ import annotations

import json
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent


def main(argv):
    if "--" in argv:
        i = argv.index("--")
        cfgs, extra = argv[:i], argv[i + 1:]
    else:
        cfgs, extra = argv, []
    for cfg in cfgs:
        cmd = [sys.executable, str(ROOT / "bench.py"), "--cpu-seconds", "0", "--overlap", cfg] + extra
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(cfg, "FAILED rc", r.returncode, r.stderr[-2000:], flush=True)
            raise SystemExit(1)
        j = json.loads(r.stdout.strip().splitlines()[-1])
        ks = (j.get("roofline") or {}).get("kernel_ms_per_step", {})
        one = j.get("one_stream") or {}
        print(f"{cfg:10s} {j['value']:9.0f} /s  {j['ms_per_step']:.3f} ms  {ks}  "
              f"one-stream {one.get('ms_per_step', float('nan')):.3f} ms  "
              f"matches {j.get('mean_stereo_matches')}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
