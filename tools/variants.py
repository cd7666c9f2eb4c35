"""A/B builds of liborbx.so from different source trees, each timed by bench.py in its own
process (ORBX_LIB selects the library).  A variant is a git revision of csrc/ + include/, or
WORK for the working tree; the product library has no compile-time variant switches.

    python tools/variants.py build base=HEAD new=WORK     # here, on the CPU
    python tools/variants.py run [bench args...]          # on the GPU box

`build` writes my_orb_slam2_amd/liborbx_<NAME>.so (git-ignored, travels with gpurun) and
tools/_variants.json; `run` prints one line per variant with pairs/s and per-kernel ms,
interleaving the variants over --rounds R (default 2) to spread box drift over all of them."""
from __future__ import annotations

import json
import os
import pathlib
import shutil
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
LIST = ROOT / "tools" / "_variants.json"


def _tree(rev: str, dst: pathlib.Path) -> pathlib.Path:
    """csrc/ and include/ of `rev` (or the working tree) under dst; returns dst/csrc."""
    for sub in ("my_orb_slam2_amd/csrc", "include"):
        if rev == "WORK":
            shutil.copytree(ROOT / sub, dst / sub)
        else:
            (dst / sub).mkdir(parents=True)
            files = subprocess.run(["git", "ls-tree", "--name-only", f"{rev}:{sub}"], cwd=ROOT,
                                   check=True, capture_output=True, text=True).stdout.split()
            for f in files:
                data = subprocess.run(["git", "show", f"{rev}:{sub}/{f}"], cwd=ROOT, check=True,
                                      capture_output=True).stdout
                (dst / sub / f).write_bytes(data)
    return dst / "my_orb_slam2_amd" / "csrc"


def build(specs):
    from my_orb_slam2_amd import build as b
    out, procs = {}, []
    for old in b.PKG.glob("liborbx_*.so"):   # stale variants would travel with every gpurun
        old.unlink()
    tmp = pathlib.Path(tempfile.mkdtemp())
    try:
        for spec in specs:
            name, _, rev = spec.partition("=")
            csrc = _tree(rev or "WORK", tmp / name)
            lib = b.PKG / f"liborbx_{name}.so"
            flags = [f for f in b.FLAGS if not f.startswith("-I")] + ["-I" + str(tmp / name / "include")]
            srcs = [str(csrc / s) for s in b.SOURCES if (csrc / s).exists()]
            # the tree's source hash, so the test fixture accepts a variant (ORBX_LIB=...)
            cmd = [b.hipcc()] + flags + [f'-DORBX_SRC_HASH="{b.source_hash()}"'] + srcs + ["-o", str(lib)]
            procs.append((name, subprocess.Popen(cmd)))
            out[name] = {"lib": str(lib.relative_to(ROOT)), "rev": rev or "WORK"}
        for name, p in procs:
            if p.wait() != 0:
                raise SystemExit(f"variant {name} failed to build")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    json.dump(out, open(LIST, "w"), indent=1)
    print("built", ", ".join(out))


def run(bench_args):
    rounds = 2
    if "--rounds" in bench_args:
        i = bench_args.index("--rounds")
        rounds = int(bench_args[i + 1])
        bench_args = bench_args[:i] + bench_args[i + 2:]
    variants = json.load(open(LIST))
    for rep in range(rounds):
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
            extra = {k: j[k] for k in ("mean_stereo_matches", "mean_keypoints_left", "verified") if k in j}
            print(f"{rep} {name:14s} {j['value']:9.0f} /s  {j['ms_per_step']:.3f} ms  {ks}  {extra}",
                  flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        run(sys.argv[2:])
