"""A/B builds of liborbx.so: the same sources compiled with different -D knobs, each timed by
bench.py in its own process (ORBX_LIB selects the library).

    python tools/variants.py build NAME=-DFOO=1,-DBAR=2 NAME2=...   # here, on the CPU
    python tools/variants.py run [bench args...]                   # on the GPU box

`build` writes my_orb_slam2_amd/liborbx_<NAME>.so (git-ignored, travels with gpurun) and
tools/_variants.json; `run` prints one line per variant with pairs/s and per-kernel ms."""
from __future__ import annotations

import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
LIST = ROOT / "tools" / "_variants.json"


def build(specs):
    from my_orb_slam2_amd import build as b
    out = {}
    procs = []
    for old in b.PKG.glob("liborbx_*.so"):   # stale variants would travel with every gpurun
        old.unlink()
    for spec in specs:
        name, _, defs = spec.partition("=")
        flags = [d for d in defs.split(",") if d]
        lib = b.PKG / f"liborbx_{name}.so"
        srcs = [str(b.CSRC / s) for s in b.SOURCES]
        # the tree's source hash too, so the test fixture accepts a variant (ORBX_LIB=...)
        cmd = ([b.hipcc()] + b.FLAGS + flags + [f'-DORBX_SRC_HASH="{b.source_hash()}"'] + srcs +
               ["-o", str(lib)])
        procs.append((name, subprocess.Popen(cmd)))
        out[name] = {"lib": str(lib.relative_to(ROOT)), "flags": flags}
    for name, p in procs:
        if p.wait() != 0:
            raise SystemExit(f"variant {name} failed to build")
    json.dump(out, open(LIST, "w"), indent=1)
    print("built", ", ".join(out))


def run(bench_args):
    variants = json.load(open(LIST))
    for name, v in variants.items():
        env = dict(os.environ, ORBX_LIB=str(ROOT / v["lib"]))
        cmd = [sys.executable, str(ROOT / "bench.py"), "--cpu-seconds", "0"] + bench_args
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(name, "FAILED rc", r.returncode, r.stderr[-2000:], flush=True)
            raise SystemExit(1)
        j = json.loads(r.stdout.strip().splitlines()[-1])
        ks = (j.get("roofline") or {}).get("one_stream_ms_per_step") or \
            (j.get("roofline") or {}).get("kernel_ms_per_step", {})
        extra = {k: j[k] for k in ("mean_stereo_matches", "mean_keypoints_left") if k in j}
        print(f"{name:14s} {j['value']:9.0f} /s  {j['ms_per_step']:.3f} ms  {ks}  {extra}",
              flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(sys.argv[2:])
