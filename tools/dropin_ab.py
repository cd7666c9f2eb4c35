"""A/B of the drop-in host path's small-batch policies (run on the GPU box).

Runs tests/native/facade_test `bench` (the facade loop) against a tuning build of liborbx.so
(tools/_var/tune/liborbx.so, built with -DORBX_TUNING, which reads the ORBX_* overrides of
orbx_capi.hip) for each setting and K, and prints median / mean latency and pairs/s.
    python tools/dropin_ab.py build            # here (hipcc)
    python tools/dropin_ab.py run DIR [K,..]   # on the box, DIR from tools/dropin_data.py
"""
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
VAR = ROOT / "tools" / "_var" / "tune"

SETTINGS = {   # "_args": extra arguments of the bench program (facade_test: "frame")
    "default": {},
    "frame": {"_args": "frame"},
    "frame_solo": {"_args": "frame", "ORBX_FRAME_SERVER": "0"},
    "frame_nochain": {"_args": "frame", "ORBX_CHAIN_MAX_BATCH": "0"},
    "frame_chain2": {"_args": "frame", "ORBX_CHAIN_MAX_BATCH": "2"},
    "frame_chain4": {"_args": "frame", "ORBX_CHAIN_MAX_BATCH": "4"},
    "frame_chain8": {"_args": "frame", "ORBX_CHAIN_MAX_BATCH": "8"},
    "frame_nostage": {"_args": "frame", "ORBX_STAGE_THREAD": "0"},
    "frame_stage2": {"_args": "frame", "ORBX_STAGE_THREAD": "2"},
    "frame_nograph": {"_args": "frame", "ORBX_EXTRACT_GRAPH": "0"},
    "frame_if1": {"_args": "frame", "ORBX_FS_INFLIGHT": "1"},
    "frame_oct16": {"_args": "frame", "ORBX_OCT_SMALL_BATCH": "16"},
    "frame_if3": {"_args": "frame", "ORBX_FS_INFLIGHT": "3"},
    "frame_q16": {"_args": "frame", "GPU_MAX_HW_QUEUES": "16"},
    "frame_side": {"_args": "frame", "ORBX_SIDE_MIN_BATCH": "1"},
    "frame_th16": {"_args": "frame", "ORBX_STRIP_TH": "16,16,16,16,16,16,16,16"},
    "frame_th32": {"_args": "frame", "ORBX_STRIP_TH": "32,32,32,32,32,32,32,32"},
    "nospin": {"ORBX_WAIT_SPIN_US": "0"},
    "nograph": {"ORBX_EXTRACT_GRAPH": "0"},
    "q16": {"GPU_MAX_HW_QUEUES": "16"},
}


def build():
    from my_orb_slam2_amd import build as b
    VAR.mkdir(parents=True, exist_ok=True)
    srcs = [str(b.CSRC / s) for s in b.SOURCES]
    cmd = ([b.hipcc()] + b.FLAGS + ["-DORBX_TUNING", f'-DORBX_SRC_HASH="{b.source_hash()}"'] +
           srcs + ["-o", str(VAR / "liborbx.so")])
    subprocess.run(cmd, check=True)
    print(VAR / "liborbx.so")


def run(d, ks):
    # the facade loop (bench.py --workload dropin's default), or ORBX_AB_BIN=boundary_test
    binp = ROOT / "tests" / "native" / os.environ.get("ORBX_AB_BIN", "facade_test")
    only = os.environ.get("ORBX_AB_SETTINGS")   # comma-separated subset of SETTINGS
    for name, env_set in SETTINGS.items():
        if only and name not in only.split(","):
            continue
        for K in ks:
            extra = env_set.get("_args", "").split()
            env = dict(os.environ, LD_LIBRARY_PATH=str(VAR),
                       **{k: v for k, v in env_set.items() if not k.startswith("_")})
            frames = 200 if K == 1 else 100
            r = subprocess.run([str(binp), "bench", d, str(frames), "20", str(K)] + extra,
                               env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(name, K, "FAILED", r.stderr[-1000:], flush=True)
                raise SystemExit(1)
            j = json.loads(r.stdout.strip().splitlines()[-1])
            v = sorted(j["latency_ms"])
            print(f"{name:10s} K={K}  median {v[len(v) // 2]:.3f} ms  mean {sum(v) / len(v):.3f} ms"
                  f"  {K * frames / (j['wall_ms'] / 1000):8.0f} pairs/s  agree "
                  f"{len(set(j['digests'])) == 1}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(sys.argv[2], [int(k) for k in (sys.argv[3] if len(sys.argv) > 3 else "1,8").split(",")])
